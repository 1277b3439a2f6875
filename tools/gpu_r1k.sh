#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 300 python tools/grad_diag.py > gpurun_out/graddiag_r1k.log 2>&1; echo "diag rc=$?"; cat gpurun_out/graddiag_r1k.log
TAG=r1k bash tools/gpu_ablate.sh || exit $?
TAG=r1k PYTEST_ARGS="tests/test_gpu_ops.py" bash tools/gpu_quick.sh
