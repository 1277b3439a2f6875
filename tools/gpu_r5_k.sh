#!/bin/bash
# Round 5: dead compile-time variants removed (CONV_BDMA / WG_SWZ / WG_FILL / HEAD_ABL / occupancy knobs as
# constants): bit identity vs abl/libprev.so (HEAD's sources) + op and debug-build tests
set -u
mkdir -p gpurun_out
timeout -k 10 300 python tools/bitcmp.py enhanced-unet_amd/eunet/libeunet_hip.so abl/libprev.so > gpurun_out/r5k_bitcmp.txt 2>&1 || { echo "bitcmp failed"; tail -5 gpurun_out/r5k_bitcmp.txt; exit 1; }
tail -2 gpurun_out/r5k_bitcmp.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_debug.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5k_pytest.log 2>&1 || { echo "pytest failed"; grep -E "^E |FAILED" gpurun_out/r5k_pytest.log | head; exit 1; }
tail -1 gpurun_out/r5k_pytest.log
echo done
