#!/bin/bash
# Round 5: kernel-boundary gaps -- rocprofv3 kernel traces of the bench step with the LDS attribute set once per
# kernel (in-tree) and per launch (abl/libprev.so); then a bench A/B
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in base prev; do
  L=""; [ $v != base ] && L=abl/lib$v.so
  EUNET_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_r5q_$v -o run -- \
    python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg --no-dual-leg > gpurun_out/prof_r5q_$v.log 2>&1 || { echo "prof failed $v"; tail -5 gpurun_out/prof_r5q_$v.log; exit 1; }
  echo "prof $v ok"
done
VARIANTS='base|env:EUNET_LIB=abl/libprev.so' ROUNDS=${ROUNDS:-2} TAG=r5q bash tools/gpu_ab_knobs.sh
