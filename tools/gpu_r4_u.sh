#!/bin/bash
# round 4: native clip + AdamW with torch's fused-AdamW precisions (in-tree build): parity tests,
# Trainer-level tests, kernel times of the optimizer tail, alternating bench native / torch path
set -u
export TMPDIR=/tmp
TAG=optim TLIM=300 bash tools/gpu_run_tests.sh tests/test_gpu_optim.py || exit $?
TAG=model TLIM=900 bash tools/gpu_run_tests.sh tests/test_gpu_model.py tests/test_gpu_configs.py tests/test_dp_gpu.py || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4u_opt -o r4u -- \
  python bench.py --steps 5 --warmup 3 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg \
  > gpurun_out/r4u_prof.log 2>&1 || exit $?
B="--steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg"
for K in 1 0 1 0 1 0; do
  timeout -k 10 300 python tools/bench_trainer_attr.py native_clip_adamw=$K -- $B > gpurun_out/r4u_bench.log 2>&1 || exit $?
  echo "bench native_clip_adamw=$K $(grep -o '"value": [0-9.]*' gpurun_out/r4u_bench.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4u_bench.log | head -1)"
done
