#!/bin/bash
# Same-box A/B of an HBM-bound kernel change: the op tests (KSEL), the step digest of both builds
# (tools/bitcmp.py), standalone timings (tools/time_memk.py, alternating), then alternating bench rounds.
# usage: LIB_B=abl/libprev.so KSEL="pool_up or row_sweep" bash tools/gpu_ab_memk.sh
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q --timeout 200 \
  --timeout-method thread -k "${KSEL}" > gpurun_out/pt_memk.log 2>&1 || { echo "pytest failed"; tail -20 gpurun_out/pt_memk.log; exit 1; }
tail -1 gpurun_out/pt_memk.log
timeout -k 10 300 python tools/bitcmp.py "" $LIB_B > gpurun_out/bitcmp_memk.log 2>&1 || { echo bitcmp fail; exit 1; }
tail -2 gpurun_out/bitcmp_memk.log
for L in "" "$LIB_B" "" "$LIB_B"; do
  EUNET_LIB=$L timeout -k 10 120 python tools/time_memk.py > gpurun_out/tm_memk.log 2>&1 || { echo tm fail; tail -3 gpurun_out/tm_memk.log; exit 1; }
  echo "[${L:-intree}] $(grep total gpurun_out/tm_memk.log | tr '\n' '|')"
done
A="" B="EUNET_LIB=$LIB_B" ROUNDS=${ROUNDS:-3} bash tools/gpu_ab_env.sh
