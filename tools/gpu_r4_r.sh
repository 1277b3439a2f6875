#!/bin/bash
# round 4: two-stage bn_finalize with additive shifted moments (abl/libbf2.so = in-tree build): op + model
# tests, kernel times, alternating bench against the one-launch bn_finalize (EUNET_BN_FINALIZE_ONE_LAUNCH=1)
set -u
export TMPDIR=/tmp
EUNET_LIB=abl/libbf2.so TAG=ops TLIM=600 bash tools/gpu_run_tests.sh tests/test_gpu_ops.py || exit $?
EUNET_LIB=abl/libbf2.so TAG=model TLIM=900 bash tools/gpu_run_tests.sh tests/test_gpu_model.py || exit $?
EUNET_LIB=abl/libbf2.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4r_bf2 -o r4r -- \
  python bench.py --steps 5 --warmup 3 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg \
  > gpurun_out/r4r_prof_bf2.log 2>&1 || exit $?
B="--steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg"
for E in 0 1 0 1 0 1 0 1; do
  EUNET_BN_FINALIZE_ONE_LAUNCH=$E EUNET_LIB=abl/libbf2.so timeout -k 10 300 python bench.py $B > gpurun_out/r4r_bench.log 2>&1 || exit $?
  echo "bench one_launch=$E $(grep -o '"value": [0-9.]*' gpurun_out/r4r_bench.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4r_bench.log | head -1)"
done
