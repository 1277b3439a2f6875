#!/bin/bash
# conv3x3 forward ablation on a few layer shapes (each run bounded)
set -u
mkdir -p gpurun_out
TAG=${TAG:-abl}
for s in "4 128 128 512 512" "4 256 256 256 256" "4 512 512 128 128" "4 1024 1024 64 64"; do
  timeout -k 10 120 tools/conv_ablate $s 10 >> gpurun_out/ablate_${TAG}.log 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "ablate rc=$rc on $s"; cat gpurun_out/ablate_${TAG}.log; exit $rc; fi
done
cat gpurun_out/ablate_${TAG}.log
