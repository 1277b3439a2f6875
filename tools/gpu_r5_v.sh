#!/bin/bash
# Round 5: the tail co-block's half-width forward / data-gradient loop (a second copy of the K loop, chosen per
# block): alternating bench runs with the fp32 and dual-branch legs, in-tree vs HEAD (abl/libprev.so)
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "conv" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r5v_pytest.log 2>&1 || { echo "pytest failed"; grep -E "^E |FAILED" gpurun_out/r5v_pytest.log | head -20; exit 1; }
tail -1 gpurun_out/r5v_pytest.log
out=gpurun_out/ab_r5v.jsonl; : > $out
for r in 1 2 3; do
  for v in base prev; do
    L=""; [ $v != base ] && L=abl/lib$v.so
    timeout -k 10 500 env ${L:+EUNET_LIB=$L} python bench.py --steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 > gpurun_out/ab_r5v_run.log 2>&1 || { echo "bench failed $v"; tail -5 gpurun_out/ab_r5v_run.log; exit 1; }
    line=$(grep '^{' gpurun_out/ab_r5v_run.log | tail -1)
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(json.dumps({'variant': sys.argv[2], 'round': int(sys.argv[3]), 'value': d['value'], 'fp32': d['fp32_configs1']['value'], 'dual': d['dual_configs4']['value']}))" "$line" "$v" "$r" >> $out
    tail -1 $out
  done
done
