#!/bin/bash
# dual-branch gradient tests under each library in LIBS ("cur" = the in-tree build)
set -u
mkdir -p gpurun_out
for L in ${LIBS:-cur}; do
  t=$(basename $L .so)
  if [ "$L" = cur ]; then
    timeout -k 10 300 python -u -m pytest tests/test_gpu_dual.py -m gpu -q -s --timeout 200 --timeout-method thread -k "${KSEL:-grads}" > gpurun_out/dab_$t.log 2>&1
  else
    EUNET_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_dual.py -m gpu -q -s --timeout 200 --timeout-method thread -k "${KSEL:-grads}" > gpurun_out/dab_$t.log 2>&1
  fi
  rc=$?; echo "$t rc=$rc"; grep -E "passed|failed" gpurun_out/dab_$t.log
  [ $rc -gt 1 ] && exit $rc
done
exit 0
