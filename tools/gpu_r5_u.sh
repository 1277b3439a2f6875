#!/bin/bash
# Round 5: skip the MFMAs of co tiles 2, 3 in the tail co-block of 96 / 288-channel layers (base 96, configs[4]),
# forward / data gradient / weight gradient, by uniform branches: conv op tests, standalone 13 layers (base 64:
# no tail block, so this is the branches' cost), then alternating bench runs with the dual-branch leg
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "conv" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r5u_pytest.log 2>&1 || { echo "pytest failed"; grep -E "^E |FAILED" gpurun_out/r5u_pytest.log | head -20; exit 1; }
tail -1 gpurun_out/r5u_pytest.log
for v in base prev; do
  L=""; [ $v != base ] && L=abl/lib$v.so
  timeout -k 10 150 env ${L:+EUNET_LIB=$L} python tools/conv_bench.py --transform --reps 10 > gpurun_out/cb_r5u_$v.log 2>&1 || { echo "cb failed $v"; tail -3 gpurun_out/cb_r5u_$v.log; exit 1; }
  echo "$v $(grep summary gpurun_out/cb_r5u_$v.log)"
done
out=gpurun_out/ab_r5u.jsonl; : > $out
for r in 1 2; do
  for v in base prev; do
    L=""; [ $v != base ] && L=abl/lib$v.so
    timeout -k 10 400 env ${L:+EUNET_LIB=$L} python bench.py --steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg > gpurun_out/ab_r5u_run.log 2>&1 || { echo "bench failed $v"; tail -5 gpurun_out/ab_r5u_run.log; exit 1; }
    line=$(grep '^{' gpurun_out/ab_r5u_run.log | tail -1)
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(json.dumps({'variant': sys.argv[2], 'round': int(sys.argv[3]), 'value': d['value'], 'dual': d['dual_configs4']['value'], 'dual_frac': d['dual_configs4']['roofline']['frac']}))" "$line" "$v" "$r" >> $out
    tail -1 $out
  done
done
