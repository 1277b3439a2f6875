#!/bin/bash
# Same-box A/B of the in-tree library against another build (LIB_B, e.g. abl/libold.so): GPU tests of the
# touched kernels (TESTS / KSEL), per-layer conv timings of both, then alternating full-bench rounds.
set -u
mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest ${TESTS} -x -q --timeout 200 --timeout-method thread ${KSEL:+-k "$KSEL"} \
    > gpurun_out/pt_ab.log 2>&1 || { echo "pytest failed"; grep -E "^E |FAILED" gpurun_out/pt_ab.log | head -20; exit 1; }
  tail -1 gpurun_out/pt_ab.log
fi
for L in "" "EUNET_LIB=$LIB_B"; do
  env $L timeout -k 10 120 python tools/conv_bench.py --transform --reps 10 > gpurun_out/cb_ab.log 2>&1 || { echo cb fail; tail -5 gpurun_out/cb_ab.log; exit 1; }
  echo "== [$L] $(grep summary gpurun_out/cb_ab.log)"
done
A="" B="EUNET_LIB=$LIB_B" ROUNDS=${ROUNDS:-3} bash tools/gpu_ab_env.sh
