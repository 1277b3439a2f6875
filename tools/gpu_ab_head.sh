#!/bin/bash
# Same-box A/B of a head change: the head GPU tests, a bit-identity digest of the in-tree library against
# LIB_B (tools/bitcmp.py), then per-kernel head times of both (tools/gpu_head_libs.sh, twice).
# usage: LIB_B=abl/libprev.so TAG=name bash tools/gpu_ab_head.sh
set -u
mkdir -p gpurun_out
TAG=${TAG:-hab}
TAG=$TAG TLIM=400 bash tools/gpu_run_tests.sh tests -m gpu -k "${KSEL:-head}" || exit $?
timeout -k 10 300 python tools/bitcmp.py "" $LIB_B > gpurun_out/bitcmp_$TAG.log 2>&1 || { echo bitcmp fail; tail -5 gpurun_out/bitcmp_$TAG.log; exit 1; }
tail -3 gpurun_out/bitcmp_$TAG.log
TAG=${TAG}1 LIBS="$LIB_B" REPS=10 bash tools/gpu_head_libs.sh || exit $?
TAG=${TAG}2 LIBS="$LIB_B" REPS=10 bash tools/gpu_head_libs.sh || exit $?
