#!/bin/bash
# Round 5: wgrad co-tail launch (NCT = 2) + dead-wave skip: tests, then A/B vs abl/libprev.so (HEAD's conv3x3)
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_dual.py tests/test_gpu_configs.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5h_pytest.log 2>&1 || { echo "pytest failed"; grep -E "^E |FAILED" gpurun_out/r5h_pytest.log | head; exit 1; }
tail -1 gpurun_out/r5h_pytest.log
: > gpurun_out/r5h_ab.txt
for r in 1 2; do
  for L in "" "EUNET_LIB=abl/libprev.so"; do
    env $L timeout -k 10 300 python3 bench.py --dual --base 96 --size 2048 --batch 2 --steps 10 --warmup 3 --no-cpu-baseline --dice-size 0 > gpurun_out/r5h_run.log 2>&1 || { echo "dual fail [$L]"; tail -5 gpurun_out/r5h_run.log; exit 1; }
    echo "dual [$L] $(grep '^{' gpurun_out/r5h_run.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"])')" | tee -a gpurun_out/r5h_ab.txt
    env $L timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg --no-dual-leg > gpurun_out/r5h_run.log 2>&1 || { echo "base fail [$L]"; tail -5 gpurun_out/r5h_run.log; exit 1; }
    echo "base [$L] $(grep '^{' gpurun_out/r5h_run.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"])')" | tee -a gpurun_out/r5h_ab.txt
  done
done
echo done
