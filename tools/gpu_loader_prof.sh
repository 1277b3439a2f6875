#!/bin/bash
# rocprofv3 kernel stats of the f2 loader alone (tools/loader_bench.py --loader-only): the device time
# one batch of the augmentation pipeline costs.  Writes gpurun_out/loader_prof_<TAG>/ and a summary.
set -u
mkdir -p gpurun_out
TAG=${TAG:-lp}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/loader_prof_${TAG} -o run -- \
  python tools/loader_bench.py --loader-only > gpurun_out/loader_prof_${TAG}.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -2 gpurun_out/loader_prof_${TAG}.log; [ $rc -ne 0 ] && exit $rc
f=$(find gpurun_out/loader_prof_${TAG} -name '*kernel_stats.csv' | head -1)
python3 tools/kstats.py "$f" 68 40 > gpurun_out/loader_prof_${TAG}.txt 2>&1 || true
head -40 gpurun_out/loader_prof_${TAG}.txt
