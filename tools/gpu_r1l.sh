#!/bin/bash
set -u
mkdir -p gpurun_out
TAG=r1l bash tools/gpu_ablate.sh || exit $?
timeout -k 10 300 python tools/grad_diag.py > gpurun_out/graddiag_r1l.log 2>&1; echo "diag rc=$?"; cat gpurun_out/graddiag_r1l.log
TAG=r1l bash tools/gpu_quick.sh
