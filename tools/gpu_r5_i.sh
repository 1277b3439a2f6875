#!/bin/bash
# Round 5: packed-fp32 bnrelu_up / up_bwd_rows: op + model tests, bit identity vs abl/libprev.so (HEAD's
# bn_pool_up), then alternating bench A/B
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -k "up or pool or bn or train_grads or bf16 or schedule" > gpurun_out/r5i_pytest.log 2>&1 || { echo "pytest failed"; grep -E "^E |FAILED" gpurun_out/r5i_pytest.log | head; exit 1; }
tail -1 gpurun_out/r5i_pytest.log
grep -E "head parameter gradients" gpurun_out/r5i_pytest.log || true
timeout -k 10 300 python tools/bitcmp.py enhanced-unet_amd/eunet/libeunet_hip.so abl/libprev.so > gpurun_out/r5i_bitcmp.txt 2>&1 || { echo "bitcmp failed"; tail -5 gpurun_out/r5i_bitcmp.txt; exit 1; }
cat gpurun_out/r5i_bitcmp.txt | tail -3
A="" B="EUNET_LIB=abl/libprev.so" ROUNDS=3 bash tools/gpu_ab_env.sh
echo done
