#!/bin/bash
# round 4: UNetEngine.fork_once (one event for the side stream's three waits after each BN-a backward):
# schedule exactness test, kernel trace (launch-stream gaps), alternating bench fork_once=1/0
set -u
export TMPDIR=/tmp
TAG=sched TLIM=400 bash tools/gpu_run_tests.sh tests/test_gpu_model.py -k "schedule or step_graph" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4ac -o r4ac -- \
  python bench.py --steps 5 --warmup 3 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg \
  > gpurun_out/r4ac_prof.log 2>&1 || exit $?
B="--steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg"
for K in 1 0 1 0 1 0 1 0; do
  timeout -k 10 300 python tools/bench_knob.py fork_once=$K -- $B > gpurun_out/r4ac_bench.log 2>&1 || exit $?
  echo "bench fork_once=$K $(grep -o '"value": [0-9.]*' gpurun_out/r4ac_bench.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4ac_bench.log | head -1)"
done
