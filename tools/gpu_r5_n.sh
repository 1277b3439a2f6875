#!/bin/bash
# Round 5: conv epilogue from registers -- conv op tests of the in-tree build, per-layer standalone timing vs
# abl/libprev.so (HEAD's LDS-staged epilogue) with the fused and the plain data gradient (per-layer lines in
# gpurun_out/cb_r5n_<variant>.log), then the bench A/B
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "conv" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r5n_pytest.log 2>&1 || { echo "pytest failed"; grep -E "^E |FAILED|Error" gpurun_out/r5n_pytest.log | head -30; exit 1; }
tail -1 gpurun_out/r5n_pytest.log
for v in base prev; do
  L=""; [ $v != base ] && L=abl/lib$v.so
  for mode in "" "--plain-dgrad --no-stats"; do
    tag=${v}$( [ -n "$mode" ] && echo _plain )
    timeout -k 10 150 env ${L:+EUNET_LIB=$L} python tools/conv_bench.py --transform --reps 10 $mode > gpurun_out/cb_r5n_$tag.log 2>&1 || { echo "cb failed $tag"; tail -3 gpurun_out/cb_r5n_$tag.log; exit 1; }
    echo "$tag $(grep summary gpurun_out/cb_r5n_$tag.log)"
  done
done
VARIANTS='base|env:EUNET_LIB=abl/libprev.so' ROUNDS=${ROUNDS:-2} TAG=r5n bash tools/gpu_ab_knobs.sh
