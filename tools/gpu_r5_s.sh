#!/bin/bash
# Round 5: SQ counters of every kernel of the bench step (tools/gpu_pmc_sq.sh); the small-conv weight gradient's
# bias sums from registers (in-tree; bit-identity vs abl/libprev.so); the small-conv forward's BN partials from
# shifted sums instead of a per-pixel Welford update (abl/libsf.so: op tests); bench A/B of the three
set -u
mkdir -p gpurun_out
TAG=r5sq PROG="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --dice-size 0 --no-fp32-leg --no-dual-leg --no-dp-world1" bash tools/gpu_pmc_sq.sh > gpurun_out/r5sq.txt 2>&1 || { echo "sq failed"; tail -5 gpurun_out/r5sq.txt; exit 1; }
echo "sq ok"
timeout -k 10 200 python tools/bitcmp.py enhanced-unet_amd/eunet/libeunet_hip.so abl/libprev.so > gpurun_out/r5s_bitcmp.log 2>&1 || { echo "bitcmp failed"; tail -5 gpurun_out/r5s_bitcmp.log; exit 1; }
cat gpurun_out/r5s_bitcmp.log
EUNET_LIB=abl/libsf.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q -k "small or stats or train_grads" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r5s_pytest.log 2>&1 || { echo "pytest failed"; grep -E "^E |FAILED" gpurun_out/r5s_pytest.log | head -20; exit 1; }
tail -1 gpurun_out/r5s_pytest.log
VARIANTS='base|env:EUNET_LIB=abl/libprev.so|env:EUNET_LIB=abl/libsf.so' ROUNDS=${ROUNDS:-2} TAG=r5s bash tools/gpu_ab_knobs.sh
