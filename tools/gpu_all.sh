#!/bin/bash
# tests -> rocprof bench -> per-layer conv bench -> grad diag (each bounded; stop on crash codes)
set -u
TAG=${TAG:-all}
SKIP_BENCH=1 TAG=$TAG bash tools/gpu_check.sh; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
TAG=$TAG bash tools/gpu_prof.sh; rc=$?
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/conv_bench.py ${CONV_ARGS:-} > gpurun_out/conv_${TAG}.log 2>&1
rc=$?; echo "conv_bench rc=$rc"; tail -1 gpurun_out/conv_${TAG}.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/grad_diag.py > gpurun_out/graddiag_${TAG}.log 2>&1; echo "grad_diag rc=$?"; head -6 gpurun_out/graddiag_${TAG}.log
