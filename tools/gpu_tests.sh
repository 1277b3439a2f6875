#!/bin/bash
# selected GPU test files (TESTS), verbose, bounded; then optional quick bench (BENCH=1)
set -u
mkdir -p gpurun_out
TAG=${TAG:-t}
timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest ${TESTS:-tests} -m gpu -v --timeout 200 --timeout-method thread \
  -rf ${PYTEST_ARGS:-} > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_${TAG}.log | tail -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ "${BENCH:-0}" = "1" ]; then
  timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench_${TAG}.log 2>&1
  brc=$?; echo "bench rc=$brc"; tail -2 gpurun_out/bench_${TAG}.log | cut -c1-600
  exit $brc
fi
exit $rc
