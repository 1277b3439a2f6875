#!/bin/bash
# round 4 end, part A: the full GPU test suite on the in-tree build (one process, per-test time limit)
set -u
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_final4c.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_final4c.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/pytest_final4c.log | head; exit $rc; }
exit 0
