#!/bin/bash
# round 4: up_bwd_rows (the upsample adjoint with the fused BN-b reduction, 258 registers = 1 wave / SIMD)
# compiled for 2 waves / SIMD (abl/libup2.so, 256 registers + 12 B scratch) vs abl/libbase.so: tests,
# bit identity, kernel times, alternating bench
set -u
export TMPDIR=/tmp
EUNET_LIB=abl/libup2.so TAG=up TLIM=400 bash tools/gpu_run_tests.sh tests/test_gpu_ops.py -k "upsample or fused_bn_reduce" || exit $?
timeout -k 10 400 python tools/bitcmp.py abl/libbase.so abl/libup2.so || exit $?
for L in base up2; do
  EUNET_LIB=abl/lib$L.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4aa_$L -o r4aa -- \
    python bench.py --steps 5 --warmup 3 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg \
    > gpurun_out/r4aa_prof_$L.log 2>&1 || exit $?
done
B="--steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg"
for L in base up2 base up2 base up2 base up2; do
  EUNET_LIB=abl/lib$L.so timeout -k 10 300 python bench.py $B > gpurun_out/r4aa_bench.log 2>&1 || exit $?
  echo "bench lib=$L $(grep -o '"value": [0-9.]*' gpurun_out/r4aa_bench.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4aa_bench.log | head -1)"
done
