#!/bin/bash
# Round 5: conv epilogue from registers (C^T MFMA layout, perm_co-packed weights): conv op + model parity tests,
# then same-box A/B against HEAD's conv3x3 (abl/libprev.so), headline and fp32 legs
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r5m_pytest.log 2>&1 || { echo "pytest failed"; grep -E "^E |FAILED|Error" gpurun_out/r5m_pytest.log | head -30; tail -5 gpurun_out/r5m_pytest.log; exit 1; }
tail -2 gpurun_out/r5m_pytest.log
VARIANTS='base|env:EUNET_LIB=abl/libprev.so' ROUNDS=3 TAG=r5m bash tools/gpu_ab_knobs.sh
