#!/bin/bash
# Round bench: full default bench (with cpu_baseline), its rocprofv3 stats, then PMC traffic passes.
set -u
mkdir -p gpurun_out
TAG=${TAG:-full}
timeout -k 10 600 python bench.py > gpurun_out/bench_${TAG}.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench_${TAG}.log
if [ $rc -ne 0 ]; then exit $rc; fi
BENCH_ARGS="--no-cpu-baseline --dice-size 0" TAG=$TAG bash tools/gpu_prof.sh > /dev/null; rc=$?
echo "prof rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
TAG=$TAG bash tools/gpu_pmc.sh
