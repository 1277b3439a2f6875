#!/bin/bash
# round 4: bnrelu_up at 4 waves / SIMD (abl/libup4.so, 128 VGPR + 20 B scratch; 136 = 3 waves now) and
# pool_bwd_add at 4 (abl/libpb4.so, 128 + 80 B) vs abl/libbase.so (= in-tree): tests, bit identity,
# kernel times, alternating bench
set -u
export TMPDIR=/tmp
for L in up4 pb4; do
  EUNET_LIB=abl/lib$L.so TAG=t_$L TLIM=400 bash tools/gpu_run_tests.sh tests/test_gpu_ops.py -k "pool or upsample or bnrelu or fused_bn_reduce" || exit $?
done
timeout -k 10 600 python tools/bitcmp.py abl/libbase.so abl/libup4.so abl/libpb4.so || exit $?
for L in base up4 pb4; do
  EUNET_LIB=abl/lib$L.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4ab_$L -o r4ab -- \
    python bench.py --steps 5 --warmup 3 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg \
    > gpurun_out/r4ab_prof_$L.log 2>&1 || exit $?
done
B="--steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg"
for L in base up4 pb4 base up4 pb4 base up4 pb4; do
  EUNET_LIB=abl/lib$L.so timeout -k 10 300 python bench.py $B > gpurun_out/r4ab_bench.log 2>&1 || exit $?
  echo "bench lib=$L $(grep -o '"value": [0-9.]*' gpurun_out/r4ab_bench.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4ab_bench.log | head -1)"
done
