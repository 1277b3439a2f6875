#!/bin/bash
# tests -> rocprof bench -> per-layer conv bench (each step bounded; stop on crash codes)
set -u
TAG=${TAG:-all}
SKIP_BENCH=1 TAG=$TAG bash tools/gpu_check.sh; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
TAG=$TAG bash tools/gpu_prof.sh; rc=$?
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/conv_bench.py ${CONV_ARGS:-} > gpurun_out/conv_${TAG}.log 2>&1
echo "conv_bench rc=$?"; cat gpurun_out/conv_${TAG}.log | tail -16
