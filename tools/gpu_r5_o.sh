#!/bin/bash
# Round 5: forward without an operand transform (the .0 convs) staged by LDS-DMA like the plain data gradient
# (abl/libpf.so): bit-identity (tools/bitcmp.py), standalone 13 layers without the transform, bench A/B
set -u
mkdir -p gpurun_out
timeout -k 10 200 python tools/bitcmp.py enhanced-unet_amd/eunet/libeunet_hip.so abl/libpf.so > gpurun_out/r5o_bitcmp.log 2>&1 || { echo "bitcmp failed"; tail -5 gpurun_out/r5o_bitcmp.log; exit 1; }
cat gpurun_out/r5o_bitcmp.log
for v in base pf; do
  L=""; [ $v != base ] && L=abl/lib$v.so
  timeout -k 10 150 env ${L:+EUNET_LIB=$L} python tools/conv_bench.py --reps 10 > gpurun_out/cb_r5o_$v.log 2>&1 || { echo "cb failed $v"; tail -3 gpurun_out/cb_r5o_$v.log; exit 1; }
  echo "$v $(grep summary gpurun_out/cb_r5o_$v.log)"
done
VARIANTS='base|env:EUNET_LIB=abl/libpf.so' ROUNDS=${ROUNDS:-3} TAG=r5o bash tools/gpu_ab_knobs.sh
