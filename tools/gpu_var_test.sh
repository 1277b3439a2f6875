#!/bin/bash
# GPU tests under each runtime variant in VARS (";"-separated env assignments), then bench A/B
set -u
mkdir -p gpurun_out
TAG=${TAG:-vt}
IFS=';' read -ra VS <<< "${VARS:-X=0}"
for v in "${VS[@]}"; do
  env $v timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_ops.py tests/test_gpu_model.py} -m gpu -q \
    --timeout 200 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1
  rc=$?; echo "pytest ($v) rc=$rc: $(tail -1 gpurun_out/pytest_${TAG}.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  if [ $rc -eq 1 ]; then grep -E "^FAILED|^E  " gpurun_out/pytest_${TAG}.log | head -8; fi
done
CONFIGS="X=0;${VARS}" TAG=$TAG bash tools/gpu_ab.sh
