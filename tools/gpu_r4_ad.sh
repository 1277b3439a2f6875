#!/bin/bash
# round 4: colsum in one launch for <= 16 row chunks (abl/libc1.so = in-tree; same summation order as the two
# launches) vs abl/libprev.so: ops + model tests, bit identity, kernel trace, alternating bench
set -u
export TMPDIR=/tmp
EUNET_LIB=abl/libc1.so TAG=ops TLIM=600 bash tools/gpu_run_tests.sh tests/test_gpu_ops.py || exit $?
EUNET_LIB=abl/libc1.so TAG=model TLIM=600 bash tools/gpu_run_tests.sh tests/test_gpu_model.py -k "grads or schedule" || exit $?
timeout -k 10 400 python tools/bitcmp.py abl/libprev.so abl/libc1.so || exit $?
EUNET_LIB=abl/libc1.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4ad -o r4ad -- \
  python bench.py --steps 5 --warmup 3 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg \
  > gpurun_out/r4ad_prof.log 2>&1 || exit $?
B="--steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg"
for L in prev c1 prev c1 prev c1 prev c1; do
  EUNET_LIB=abl/lib$L.so timeout -k 10 300 python bench.py $B > gpurun_out/r4ad_bench.log 2>&1 || exit $?
  echo "bench lib=$L $(grep -o '"value": [0-9.]*' gpurun_out/r4ad_bench.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4ad_bench.log | head -1)"
done
