#!/bin/bash
# Round 5: head_gh with its 16 channels' BN-backward constants in VGPRs (64 registers; 2 blocks / CU) instead of
# 16 LDS b128 reads per row (abl/librc.so): bit-identity, per-kernel head times, bench A/B
set -u
mkdir -p gpurun_out
timeout -k 10 200 python tools/bitcmp.py enhanced-unet_amd/eunet/libeunet_hip.so abl/librc.so > gpurun_out/r5w_bitcmp.log 2>&1 || { echo "bitcmp failed"; tail -5 gpurun_out/r5w_bitcmp.log; exit 1; }
cat gpurun_out/r5w_bitcmp.log
TAG=r5w LIBS="abl/librc.so" bash tools/gpu_head_libs.sh > /dev/null 2>&1 || { echo "head libs failed"; exit 1; }
grep -E "==|head_gh" gpurun_out/head_libs_r5w.txt
VARIANTS='base|env:EUNET_LIB=abl/librc.so' ROUNDS=${ROUNDS:-2} TAG=r5w bash tools/gpu_ab_knobs.sh
