#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (no PMC counters here).
set -u
mkdir -p gpurun_out
TAG=${TAG:-prof}
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 ${PROF_TIMEOUT:-500} rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- \
  python bench.py ${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg --no-dual-leg} > gpurun_out/prof_${TAG}.log 2>&1
rc=$?
echo "rocprof rc=$rc"
tail -3 gpurun_out/prof_${TAG}.log
f=$(find gpurun_out/prof_${TAG} -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && head -40 "$f" | cut -c1-220
exit $rc
