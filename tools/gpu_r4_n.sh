#!/bin/bash
# round 4: wg3_early_last (the trunk's last block: conv .3's weight gradient beside conv .3's data gradient
# instead of at the step's tail) on/off, and CONV_PRIO=0 (no s_setprio around the conv MFMA phase) vs in-tree
set -u
TAG=sched TLIM=500 bash tools/gpu_run_tests.sh tests/test_gpu_model.py -k "schedule or step_graph" || exit $?
B="--steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg"
for K in 1 0 1 0 1 0; do
  timeout -k 10 300 python tools/bench_knob.py wg3_early_last=$K -- $B > gpurun_out/r4n_bench.log 2>&1 || exit $?
  echo "bench wg3_early_last=$K $(grep -o '"value": [0-9.]*' gpurun_out/r4n_bench.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4n_bench.log | head -1)"
done
LIBS="abl/libcur.so abl/libprio0.so" ROUNDS=2 bash tools/gpu_cb_libs.sh || exit $?
for L in abl/libcur.so abl/libprio0.so abl/libcur.so abl/libprio0.so; do
  EUNET_LIB=$L timeout -k 10 300 python bench.py $B > gpurun_out/r4n_bench.log 2>&1 || exit $?
  echo "bench lib=$L $(grep -o '"value": [0-9.]*' gpurun_out/r4n_bench.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4n_bench.log | head -1)"
done
