#!/bin/bash
# full GPU test suite, then the round-end measurement pass (tools/gpu_round_final.sh)
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_final3.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_final3.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/pytest_final3.log | head; exit $rc; }
TAG=${TAG:-r3b} R=r03 bash tools/gpu_round_final.sh
