#!/bin/bash
# round 4: conv A1 (the halo of an untransformed forward -- the ".0" convs -- by buffer_load ... lds too: the
# K-chunk's staging is one asynchronous round trip) vs B1+H3 (in-tree): conv parity, per-layer conv_bench, bench
set -u
EUNET_LIB=abl/liba1h3.so TAG=conv_a1 TLIM=500 bash tools/gpu_run_tests.sh tests/test_gpu_ops.py -k "conv" || exit $?
EUNET_LIB=abl/liba1h3.so TAG=model_a1 TLIM=600 bash tools/gpu_run_tests.sh tests/test_gpu_model.py tests/test_gpu_dual.py tests/test_gpu_configs.py || exit $?
LIBS="abl/libb1h3.so abl/liba1h3.so" ROUNDS=2 bash tools/gpu_cb_libs.sh || exit $?
for L in abl/libb1h3.so abl/liba1h3.so abl/libb1h3.so abl/liba1h3.so; do
  EUNET_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg > gpurun_out/r4g_bench.log 2>&1 || exit $?
  echo "bench lib=$L $(grep -o '"value": [0-9.]*' gpurun_out/r4g_bench.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4g_bench.log | head -1) $(grep -o '"encoder_fwd": {"achieved": [0-9.]*, "frac": [0-9.]*' gpurun_out/r4g_bench.log)"
done
