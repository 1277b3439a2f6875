#!/bin/bash
# GPU-box check: GPU tests, then a short bench.  Stops at the first crash-type
# exit status (fault/abort/segv/timeout) -- never retries a GPU step.
set -u
mkdir -p gpurun_out
TAG=${TAG:-run}
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -q --timeout 300 -rf \
  ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu_${TAG}.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -40 gpurun_out/pytest_gpu_${TAG}.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: pytest exit $rc"; exit $rc; fi
if [ "${SKIP_BENCH:-0}" = "1" ]; then exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py ${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu-baseline} \
  > gpurun_out/bench_${TAG}.log 2>&1
brc=$?
echo "bench rc=$brc"
tail -20 gpurun_out/bench_${TAG}.log
exit $brc
