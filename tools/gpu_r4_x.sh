#!/bin/bash
# round 4: conv_small_wgrad's x prefetch kept raw (its bf16 conversion had made every prefetch load wait in
# its bounds branch) and pack_many's loads issued before their selects (abl/libcs2.so = in-tree, on top of
# abl/libhd.so): op tests, bit identity, kernel times, alternating bench
set -u
export TMPDIR=/tmp
TAG=ops TLIM=600 bash tools/gpu_run_tests.sh tests/test_gpu_ops.py || exit $?
timeout -k 10 400 python tools/bitcmp.py abl/libhd.so abl/libcs2.so || exit $?
EUNET_LIB=abl/libcs2.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4x_cs2 -o r4x -- \
  python bench.py --steps 5 --warmup 3 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg \
  > gpurun_out/r4x_prof.log 2>&1 || exit $?
B="--steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg"
for L in hd cs2 hd cs2 hd cs2 hd cs2; do
  EUNET_LIB=abl/lib$L.so timeout -k 10 300 python bench.py $B > gpurun_out/r4x_bench.log 2>&1 || exit $?
  echo "bench lib=$L $(grep -o '"value": [0-9.]*' gpurun_out/r4x_bench.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4x_bench.log | head -1)"
done
