#!/bin/bash
# round 4: two-stage bn_finalize (abl/libbf.so, the in-tree build: + pack_many flat map + colsum batched
# loads) -- op tests, bit-identity vs the round-4 build is NOT expected (fp64 merge order); enc1.0's
# conv_small_wgrad with 768 / 1024 blocks (abl/libsw768.so, abl/libsw1024.so on top of libbf);
# kernel times; alternating bench incl. the one-launch bn_finalize knob
set -u
export TMPDIR=/tmp
EUNET_LIB=abl/libbf.so TAG=ops TLIM=600 bash tools/gpu_run_tests.sh tests/test_gpu_ops.py || exit $?
for L in sw768 sw1024; do
  EUNET_LIB=abl/lib$L.so TAG=small_$L TLIM=300 bash tools/gpu_run_tests.sh tests/test_gpu_ops.py -k "conv_small" || exit $?
done
for L in bf sw768 sw1024; do
  EUNET_LIB=abl/lib$L.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4q_$L -o r4q -- \
    python bench.py --steps 5 --warmup 3 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg \
    > gpurun_out/r4q_prof_$L.log 2>&1 || exit $?
done
B="--steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg"
for L in bf bf1 sw768 sw1024 bf bf1 sw768 sw1024 bf bf1 sw768 sw1024; do
  if [ $L = bf1 ]; then E=1; LL=bf; else E=0; LL=$L; fi
  EUNET_BN_FINALIZE_ONE_LAUNCH=$E EUNET_LIB=abl/lib$LL.so timeout -k 10 300 python bench.py $B > gpurun_out/r4q_bench.log 2>&1 || exit $?
  echo "bench lib=$L $(grep -o '"value": [0-9.]*' gpurun_out/r4q_bench.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4q_bench.log | head -1)"
done
