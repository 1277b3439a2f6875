#!/bin/bash
# Per-kernel head times (tools/head_bench.py under rocprofv3) for the in-tree library and each LIBS entry.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
out=gpurun_out/head_libs_${TAG:-h}.txt
: > $out
for L in "" ${LIBS:-}; do
  n=$(basename ${L:-intree} .so)
  EUNET_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/hb_$n -o run -- \
    python tools/head_bench.py --reps ${REPS:-10} > gpurun_out/hb_$n.log 2>&1 || { echo "fail $n"; tail -3 gpurun_out/hb_$n.log; exit 1; }
  f=$(find gpurun_out/hb_$n -name '*kernel_stats.csv' | head -1)
  echo "== $n $(tail -1 gpurun_out/hb_$n.log)" >> $out
  python3 tools/kstats.py "$f" $(( ${REPS:-10} + 2 )) 12 >> $out
done
cat $out
