#!/bin/bash
# Round 5: the strict-floor trained-model logits test, then static conv priority (odd blocks prio 1, no flips) A/B
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -q -s -k "north_star" --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/r5l_pytest.log 2>&1 || { echo "pytest failed"; grep -E "^E |FAILED|per pixel" gpurun_out/r5l_pytest.log | head; exit 1; }
grep -E "per pixel|passed" gpurun_out/r5l_pytest.log
VARIANTS='base|env:EUNET_LIB=abl/libprio.so' ROUNDS=4 TAG=r5l bash tools/gpu_ab_knobs.sh
