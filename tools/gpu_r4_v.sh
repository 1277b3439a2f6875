#!/bin/bash
# round 4: wgrad_reduce with 8 splits' loads in flight (abl/libwr.so = in-tree; same summation order) vs
# abl/libopt.so: conv tests, bit identity of two bench-size steps, kernel times, alternating bench
set -u
export TMPDIR=/tmp
TAG=optim TLIM=300 bash tools/gpu_run_tests.sh tests/test_gpu_optim.py || exit $?
TAG=conv TLIM=400 bash tools/gpu_run_tests.sh tests/test_gpu_ops.py -k "wgrad or conv_small" || exit $?
timeout -k 10 400 python tools/bitcmp.py abl/libopt.so abl/libwr.so || exit $?
EUNET_LIB=abl/libwr.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4v_wr -o r4v -- \
  python bench.py --steps 5 --warmup 3 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg \
  > gpurun_out/r4v_prof.log 2>&1 || exit $?
B="--steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg"
for L in opt wr opt wr opt wr opt wr; do
  EUNET_LIB=abl/lib$L.so timeout -k 10 300 python bench.py $B > gpurun_out/r4v_bench.log 2>&1 || exit $?
  echo "bench lib=$L $(grep -o '"value": [0-9.]*' gpurun_out/r4v_bench.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4v_bench.log | head -1)"
done
