#!/bin/bash
# Round 5: the weight gradient's half-width k loop for tail co-blocks (CT instantiation) (only the 96 / 288-channel
# layers of base 96 launch them): base-64 bit-identity vs HEAD, the dual-branch / configs[4] tests, bench with the
# dual leg, alternating
set -u
mkdir -p gpurun_out
timeout -k 10 200 python tools/bitcmp.py enhanced-unet_amd/eunet/libeunet_hip.so abl/libprev.so > gpurun_out/r5z_bitcmp.log 2>&1 || { echo "bitcmp failed"; tail -5 gpurun_out/r5z_bitcmp.log; exit 1; }
cat gpurun_out/r5z_bitcmp.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_dual.py tests/test_gpu_configs.py tests/test_gpu_ops.py -x -q -k "dual or configs4 or base96 or conv" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5z_pytest.log 2>&1 || { echo "pytest failed"; grep -E "^E |FAILED|Error" gpurun_out/r5z_pytest.log | head -20; exit 1; }
tail -1 gpurun_out/r5z_pytest.log
out=gpurun_out/ab_r5z.jsonl; : > $out
for r in 1 2 3; do
  for v in base prev; do
    L=""; [ $v != base ] && L=abl/lib$v.so
    timeout -k 10 400 env ${L:+EUNET_LIB=$L} python bench.py --steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg > gpurun_out/ab_r5z_run.log 2>&1 || { echo "bench failed $v"; tail -5 gpurun_out/ab_r5z_run.log; exit 1; }
    line=$(grep '^{' gpurun_out/ab_r5z_run.log | tail -1)
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(json.dumps({'variant': sys.argv[2], 'round': int(sys.argv[3]), 'value': d['value'], 'dual': d['dual_configs4']['value'], 'dual_frac': d['dual_configs4']['roofline']['frac']}))" "$line" "$v" "$r" >> $out
    tail -1 $out
  done
done
