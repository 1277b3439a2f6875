#!/bin/bash
# round 4: bnrelu_pool with its 2x2 window loaded before the activation stores (abl/libbp.so = in-tree) vs
# abl/libcur2.so, and the optimizer's table cache (python): tests, bit identity, kernel trace, alternating bench
set -u
export TMPDIR=/tmp
TAG=optim TLIM=300 bash tools/gpu_run_tests.sh tests/test_gpu_optim.py || exit $?
TAG=ops TLIM=600 bash tools/gpu_run_tests.sh tests/test_gpu_ops.py -k "pool or bnrelu" || exit $?
timeout -k 10 400 python tools/bitcmp.py abl/libcur2.so abl/libbp.so || exit $?
EUNET_LIB=abl/libbp.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4y_bp -o r4y -- \
  python bench.py --steps 5 --warmup 3 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg \
  > gpurun_out/r4y_prof.log 2>&1 || exit $?
B="--steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg"
for L in cur2 bp cur2 bp cur2 bp cur2 bp; do
  EUNET_LIB=abl/lib$L.so timeout -k 10 300 python bench.py $B > gpurun_out/r4y_bench.log 2>&1 || exit $?
  echo "bench lib=$L $(grep -o '"value": [0-9.]*' gpurun_out/r4y_bench.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4y_bench.log | head -1)"
done
