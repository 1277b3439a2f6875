#!/bin/bash
# round 4: phase shares of the conv forward / data-gradient blocks (stamp-instrumented diagnostic build)
set -u
mkdir -p gpurun_out
EUNET_LIB=abl/libstamp.so timeout -k 10 300 python tools/conv_stamps.py > gpurun_out/conv_stamps.txt 2>&1
rc=$?; echo "stamps rc=$rc"; cat gpurun_out/conv_stamps.txt | grep -v amdgpu.ids; exit $rc
