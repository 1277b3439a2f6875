#!/bin/bash
# head_gh variants under rocprofv3 (kernel time per launch) for the in-tree library and each LIBS entry.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for L in "" ${LIBS:-}; do
  n=$(basename ${L:-intree} .so)
  EUNET_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/hg_$n -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --dice-size 0 > gpurun_out/hg_$n.log 2>&1 || { echo "fail $n"; tail -3 gpurun_out/hg_$n.log; exit 1; }
  f=$(find gpurun_out/hg_$n -name '*kernel_stats.csv' | head -1)
  echo "$n $(grep -E 'head_gh' $f | cut -d, -f2-4 | tr '\n' ' ')"
done
