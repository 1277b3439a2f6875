#!/bin/bash
# Round 5: the dual model's first trunk hands its final weight gradient to the side stream (its split reduction
# had held the launch stream 2.4 ms waiting for CU room): dual parity tests, then bench with the dual leg vs HEAD's
# engine (git worktree of HEAD's Python package with the in-tree library)
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dual.py tests/test_dp_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5d4_pytest.log 2>&1 || { echo "pytest failed"; grep -E "^E |FAILED|Error" gpurun_out/r5d4_pytest.log | head -20; exit 1; }
tail -1 gpurun_out/r5d4_pytest.log
out=gpurun_out/ab_r5d4.jsonl; : > $out
for r in 1 2 3; do
  for v in base prev; do
    d=.; [ $v = prev ] && d=abl/prevpy
    (cd $d && timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg) > gpurun_out/ab_r5d4_run.log 2>&1 || { echo "bench failed $v"; tail -5 gpurun_out/ab_r5d4_run.log; exit 1; }
    line=$(grep '^{' gpurun_out/ab_r5d4_run.log | tail -1)
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(json.dumps({'variant': sys.argv[2], 'round': int(sys.argv[3]), 'value': d['value'], 'dual': d['dual_configs4']['value']}))" "$line" "$v" "$r" >> $out
    tail -1 $out
  done
done
