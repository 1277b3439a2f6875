#!/bin/bash
# Round 5: the weight gradient's waves whose 16 ci lie past cin skip their k-loop (base 96 tail ci-blocks) --
# bit-identity (headline step), small-conv op tests and dual tests, bench with the dual leg vs HEAD
set -u
mkdir -p gpurun_out
timeout -k 10 200 python tools/bitcmp.py enhanced-unet_amd/eunet/libeunet_hip.so abl/libprev.so > gpurun_out/r5ct_bitcmp.log 2>&1 || { echo "bitcmp failed"; tail -5 gpurun_out/r5ct_bitcmp.log; exit 1; }
cat gpurun_out/r5ct_bitcmp.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_dual.py -x -q -k "conv or dual" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5ct_pytest.log 2>&1 || { echo "pytest failed"; grep -E "^E |FAILED|Error" gpurun_out/r5ct_pytest.log | head -20; exit 1; }
tail -1 gpurun_out/r5ct_pytest.log
out=gpurun_out/ab_r5ct.jsonl; : > $out
for r in 1 2 3; do
  for v in base prev; do
    L=""; [ $v != base ] && L=abl/lib$v.so
    timeout -k 10 400 env ${L:+EUNET_LIB=$L} python bench.py --steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg > gpurun_out/ab_r5ct_run.log 2>&1 || { echo "bench failed $v"; tail -5 gpurun_out/ab_r5ct_run.log; exit 1; }
    line=$(grep '^{' gpurun_out/ab_r5ct_run.log | tail -1)
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(json.dumps({'variant': sys.argv[2], 'round': int(sys.argv[3]), 'value': d['value'], 'dual': d['dual_configs4']['value']}))" "$line" "$v" "$r" >> $out
    tail -1 $out
  done
done
