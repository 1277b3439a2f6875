#!/bin/bash
# quick GPU iteration: selected pytest (PYTEST_K), then conv_bench; each bounded.
set -u
mkdir -p gpurun_out
TAG=${TAG:-quick}
timeout -k 10 600 python -m pytest tests -m gpu -q --timeout 300 -rf ${PYTEST_ARGS:-} > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -12 gpurun_out/pytest_${TAG}.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/conv_bench.py ${CONV_ARGS:-} > gpurun_out/conv_${TAG}.log 2>&1
rc=$?; echo "conv_bench rc=$rc"; cat gpurun_out/conv_${TAG}.log | cut -c1-200
exit $rc
