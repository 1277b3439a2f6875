#!/bin/bash
# Round 5: side-stream forks / joins through eunet_stream_wait (device-scope event release) vs torch's
# wait_stream (system-scope): DP / driver tests, then a bench A/B of the engine knob, 3 rounds
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_dp_gpu.py tests/test_gpu_driver.py tests/test_gpu_dual.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r5r_pytest.log 2>&1 || { echo "pytest failed"; grep -E "^E |FAILED|Error" gpurun_out/r5r_pytest.log | head -30; exit 1; }
tail -1 gpurun_out/r5r_pytest.log
VARIANTS='base|device_fence_forks=0' ROUNDS=${ROUNDS:-3} TAG=r5r bash tools/gpu_ab_knobs.sh
