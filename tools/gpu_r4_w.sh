#!/bin/bash
# round 4: head kernels without serialized loads (abl/libhd.so = in-tree): weight fragments loaded at clamped
# indices before their selects, g_o prefetch without the 2x2-mean factor in its branch, patch gather loads
# first -- head tests, bit identity vs abl/libopt.so, kernel times, alternating bench
set -u
export TMPDIR=/tmp
TAG=head TLIM=400 bash tools/gpu_run_tests.sh tests/test_gpu_ops.py -k "head" || exit $?
timeout -k 10 400 python tools/bitcmp.py abl/libopt.so abl/libhd.so || exit $?
for L in opt hd; do
  EUNET_LIB=abl/lib$L.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4w_$L -o r4w -- \
    python bench.py --steps 5 --warmup 3 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg \
    > gpurun_out/r4w_prof_$L.log 2>&1 || exit $?
done
B="--steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg"
for L in opt hd opt hd opt hd opt hd; do
  EUNET_LIB=abl/lib$L.so timeout -k 10 300 python bench.py $B > gpurun_out/r4w_bench.log 2>&1 || exit $?
  echo "bench lib=$L $(grep -o '"value": [0-9.]*' gpurun_out/r4w_bench.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4w_bench.log | head -1)"
done
