#!/bin/bash
# Round 5: the stream-ordering test; weight-gradient blocks per launch 512 (in-tree) vs 768 / 1024
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_driver.py -x -q -k "stream_wait" --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/r5x_pytest.log 2>&1 || { echo "pytest failed"; grep -E "^E |FAILED|Error" gpurun_out/r5x_pytest.log | head -20; exit 1; }
tail -1 gpurun_out/r5x_pytest.log
VARIANTS='base|env:EUNET_LIB=abl/libwg768.so|env:EUNET_LIB=abl/libwg1024.so' ROUNDS=${ROUNDS:-2} TAG=r5x bash tools/gpu_ab_knobs.sh
