#!/bin/bash
set -u
mkdir -p gpurun_out
TAG=${TAG:-wg}
for s in "4 128 128 512 512" "4 256 256 768 256" "4 512 512 384 128" "4 1024 1024 192 64" "4 1024 1024 64 64"; do
  timeout -k 10 120 tools/conv_ablate wgrad $s 10 >> gpurun_out/ablate_wg_${TAG}.log 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "ablate rc=$rc on $s"; cat gpurun_out/ablate_wg_${TAG}.log; exit $rc; fi
done
cat gpurun_out/ablate_wg_${TAG}.log
