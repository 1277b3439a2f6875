#!/bin/bash
set -u
mkdir -p gpurun_out
TAG=${TAG:-c2}
timeout -k 10 600 python -m pytest tests/test_gpu_ops.py -q --timeout 300 -rf -k "conv3x3" > gpurun_out/pytest_conv_${TAG}.log 2>&1
rc=$?; echo "pytest conv rc=$rc"; tail -5 gpurun_out/pytest_conv_${TAG}.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/conv_bench.py > gpurun_out/conv_${TAG}.log 2>&1; echo "conv_bench rc=$?"; tail -14 gpurun_out/conv_${TAG}.log
timeout -k 10 300 python tools/grad_diag.py > gpurun_out/graddiag_${TAG}.log 2>&1; echo "grad_diag rc=$?"; head -12 gpurun_out/graddiag_${TAG}.log
