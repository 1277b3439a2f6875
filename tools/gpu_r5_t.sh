#!/bin/bash
# Round 5: weight-gradient blocks per launch (split count): 512 (in-tree) vs 256 / 384 -- half / 3/4 of the fp32
# partials written and reduced; bench A/B (the wgrad shares the chip with the launch stream)
set -u
mkdir -p gpurun_out
VARIANTS='base|env:EUNET_LIB=abl/libwg256.so|env:EUNET_LIB=abl/libwg384.so' ROUNDS=${ROUNDS:-3} TAG=r5t bash tools/gpu_ab_knobs.sh
