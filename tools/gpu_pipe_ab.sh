#!/bin/bash
# correctness of a variant library (conv op tests + whole-network gradient tests) then conv_bench A/B
set -u
mkdir -p gpurun_out
L=${LIB:-abl/libpipe.so}
EUNET_LIB=$L timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -m gpu -q -x --timeout 200 --timeout-method thread -k "${KSEL:-conv3x3 or train_grads or step}" > gpurun_out/pipe_t.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/pipe_t.log)"; [ $rc -ne 0 ] && { grep -E "^E |Error|FAILED" gpurun_out/pipe_t.log | head -10; exit $rc; }
ROUNDS=${ROUNDS:-2} CB_ARGS="${CB_ARGS:-}" LIBS="abl/libcur.so $L" bash tools/gpu_conv_ab.sh 2>&1 | grep -v "tests rc"
