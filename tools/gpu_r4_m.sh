#!/bin/bash
# round 4: epilogue sub-phase stamps of the conv kernels (abl/libstamp.so), PRY2 (plain dgrad: first-pass y
# before the last K-chunk's MFMAs, second-pass y during the first pass) vs the committed build (libcur) and
# PRY: parity of the in-tree build (PRY2), conv_bench (3 rounds), bench
set -u
mkdir -p gpurun_out
EUNET_LIB=abl/libstamp.so timeout -k 10 300 python tools/conv_stamps.py > gpurun_out/conv_stamps2.txt 2>&1 || { echo "stamps failed"; tail -5 gpurun_out/conv_stamps2.txt; exit 1; }
grep layer gpurun_out/conv_stamps2.txt
TAG=conv_pry2 TLIM=500 bash tools/gpu_run_tests.sh tests/test_gpu_ops.py -k "conv or dgrad" || exit $?
TAG=model_pry2 TLIM=700 bash tools/gpu_run_tests.sh tests/test_gpu_model.py tests/test_gpu_dual.py || exit $?
LIBS="abl/libcur.so abl/libpry.so abl/libpry2.so" ROUNDS=3 bash tools/gpu_cb_libs.sh || exit $?
for L in abl/libcur.so abl/libpry2.so abl/libcur.so abl/libpry2.so; do
  EUNET_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg > gpurun_out/r4m_bench.log 2>&1 || exit $?
  echo "bench lib=$L $(grep -o '"value": [0-9.]*' gpurun_out/r4m_bench.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4m_bench.log | head -1)"
done
