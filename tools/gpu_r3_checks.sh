#!/bin/bash
# Round-3 checks in one call: data / debug / dual bf16 / DP GPU tests, the loader benchmark, the DP trace.
set -u
mkdir -p gpurun_out
TAG=t7 NO_BENCH=1 PYTEST_TIMEOUT=900 TESTS="tests/test_gpu_data.py tests/test_gpu_debug.py tests/test_gpu_dual.py tests/test_dp_gpu.py" \
  KSEL="sync_free or prefetching or debug_build or cell_dataset or instance or bf16_train_grads or configs3" \
  bash tools/gpu_tests_bench.sh || exit $?
timeout -k 10 400 python tools/loader_bench.py > gpurun_out/loader_t7.log 2>&1 || { echo "loader bench failed"; tail -5 gpurun_out/loader_t7.log; exit 1; }
tail -2 gpurun_out/loader_t7.log
TAG=dp7 bash tools/gpu_dp_trace.sh
