#!/bin/bash
# round 4: gradient pointers as the optimizer kernels' argument (cached device table, no per-step copy) and
# dec1's 1x1 gradient column sums written straight into their slots (in-tree build): optimizer / model
# tests, kernel trace, bench
set -u
export TMPDIR=/tmp
TAG=optim TLIM=300 bash tools/gpu_run_tests.sh tests/test_gpu_optim.py || exit $?
TAG=model TLIM=900 bash tools/gpu_run_tests.sh tests/test_gpu_model.py tests/test_dp_gpu.py || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4z -o r4z -- \
  python bench.py --steps 5 --warmup 3 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg \
  > gpurun_out/r4z_prof.log 2>&1 || exit $?
B="--steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg"
for i in 1 2 3 4; do
  timeout -k 10 300 python bench.py $B > gpurun_out/r4z_bench.log 2>&1 || exit $?
  echo "bench $(grep -o '"value": [0-9.]*' gpurun_out/r4z_bench.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4z_bench.log | head -1)"
done
