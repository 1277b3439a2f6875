#!/bin/bash
# Round 5: conv epilogue with two block barriers fewer (statistics combine after the first staging barrier,
# BN-backward scratch off the staging area): conv + model tests, bit identity vs abl/libprev.so, A/B
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -q -x -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5j_pytest.log 2>&1 || { echo "pytest failed"; grep -E "^E |FAILED" gpurun_out/r5j_pytest.log | head; exit 1; }
tail -1 gpurun_out/r5j_pytest.log
grep -E "head parameter gradients" gpurun_out/r5j_pytest.log || true
timeout -k 10 300 python tools/bitcmp.py enhanced-unet_amd/eunet/libeunet_hip.so abl/libprev.so > gpurun_out/r5j_bitcmp.txt 2>&1 || { echo "bitcmp failed"; tail -5 gpurun_out/r5j_bitcmp.txt; exit 1; }
tail -2 gpurun_out/r5j_bitcmp.txt
A="" B="EUNET_LIB=abl/libprev.so" ROUNDS=3 bash tools/gpu_ab_env.sh
echo done
