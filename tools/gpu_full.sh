#!/bin/bash
# full GPU test suite, the default bench line, then a rocprofv3 --kernel-trace --stats pass of a short bench run
set -u
mkdir -p gpurun_out
TAG=${TAG:-full}
TESTS=${TESTS:-tests} TAG=$TAG PYTEST_TIMEOUT=800 BENCH_TIMEOUT=400 bash tools/gpu_tests_bench.sh || exit 1
BENCH_ARGS="--steps 10 --warmup 3 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg" TAG=$TAG bash tools/gpu_prof.sh > gpurun_out/prof_${TAG}_run.log 2>&1 || { echo "prof failed"; exit 1; }
python3 tools/kstats.py gpurun_out/prof_${TAG}/run_kernel_stats.csv 13 2>/dev/null | head -30 || true
