#!/bin/bash
# Round 5: the transformed forward (conv .3: BN+ReLU of its input in staging) by LDS-DMA too, the transform applied
# in place in LDS by the thread that loaded each slot (abl/libpt.so): bit-identity, standalone 13 layers with the
# transform, bench A/B
set -u
mkdir -p gpurun_out
timeout -k 10 200 python tools/bitcmp.py enhanced-unet_amd/eunet/libeunet_hip.so abl/libpt.so > gpurun_out/r5p_bitcmp.log 2>&1 || { echo "bitcmp failed"; tail -5 gpurun_out/r5p_bitcmp.log; exit 1; }
cat gpurun_out/r5p_bitcmp.log
for v in base pt; do
  L=""; [ $v != base ] && L=abl/lib$v.so
  timeout -k 10 150 env ${L:+EUNET_LIB=$L} python tools/conv_bench.py --transform --reps 10 > gpurun_out/cb_r5p_$v.log 2>&1 || { echo "cb failed $v"; tail -3 gpurun_out/cb_r5p_$v.log; exit 1; }
  echo "$v $(grep summary gpurun_out/cb_r5p_$v.log)"
done
VARIANTS='base|env:EUNET_LIB=abl/libpt.so' ROUNDS=${ROUNDS:-3} TAG=r5p bash tools/gpu_ab_knobs.sh
