#!/bin/bash
# eval-path GPU tests, then a short bench with the Dice-vs-CPU-reference leg.
set -u
mkdir -p gpurun_out
TAG=${TAG:-eval}
timeout -k 10 400 python -u -m pytest tests/test_gpu_eval.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_${TAG}.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_${TAG}.log 2>&1
brc=$?; echo "bench rc=$brc"; tail -3 gpurun_out/bench_${TAG}.log
exit $brc
