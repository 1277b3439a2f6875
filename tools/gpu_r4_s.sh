#!/bin/bash
# round 4: final small-kernel candidate (in-tree = abl/libnew.so: pack_many flat map, colsum / bn_finalize
# batched loads): op tests, bit identity with the committed build, alternating bench
set -u
export TMPDIR=/tmp
TAG=ops TLIM=600 bash tools/gpu_run_tests.sh tests/test_gpu_ops.py || exit $?
timeout -k 10 400 python tools/bitcmp.py abl/libcur.so abl/libnew.so || exit $?
B="--steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg"
for L in cur new cur new cur new cur new; do
  EUNET_LIB=abl/lib$L.so timeout -k 10 300 python bench.py $B > gpurun_out/r4s_bench.log 2>&1 || exit $?
  echo "bench lib=$L $(grep -o '"value": [0-9.]*' gpurun_out/r4s_bench.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4s_bench.log | head -1)"
done
