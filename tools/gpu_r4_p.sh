#!/bin/bash
# round 4: bn_finalize / colsum with their loads batched (same summation order, abl/libcs.so) and
# pack_many on a flat block map (abl/libpk.so = both): op parity tests, bit
# identity of two bench-size bf16 steps against the committed build, kernel times, alternating bench
set -u
export TMPDIR=/tmp
EUNET_LIB=abl/libpk.so TAG=ops TLIM=600 bash tools/gpu_run_tests.sh tests/test_gpu_ops.py || exit $?
timeout -k 10 400 python tools/bitcmp.py abl/libcur.so abl/libcs.so abl/libpk.so || exit $?
B="--steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg"
for L in cur pk; do
  EUNET_LIB=abl/lib$L.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4p_$L -o r4p -- \
    python bench.py --steps 5 --warmup 3 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg \
    > gpurun_out/r4p_prof_$L.log 2>&1 || exit $?
done
for L in cur cs pk cur cs pk cur cs pk; do
  EUNET_LIB=abl/lib$L.so timeout -k 10 300 python bench.py $B > gpurun_out/r4p_bench.log 2>&1 || exit $?
  echo "bench lib=$L $(grep -o '"value": [0-9.]*' gpurun_out/r4p_bench.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4p_bench.log | head -1)"
done
