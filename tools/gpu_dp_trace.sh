#!/bin/bash
# rocprofv3 kernel trace of the bench with its DataParallel (RCCL, world 1) leg last, then the step
# timeline of a DP step (tools/trace_steps.py): where the bucket all-reduce kernels land relative to
# the backward.  Writes gpurun_out/dp_trace_<TAG>.txt.
set -u
mkdir -p gpurun_out
TAG=${TAG:-dp}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- \
  python bench.py --steps 6 --warmup 2 --no-cpu-baseline --dice-size 0 --no-fp32-leg --no-dual-leg > gpurun_out/prof_${TAG}.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/prof_${TAG}.log; exit $rc; }
f=$(find gpurun_out/prof_${TAG} -name '*kernel_trace.csv' | head -1)
python3 tools/trace_steps.py "$f" 2 20 > gpurun_out/dp_trace_${TAG}.txt
grep -i -E "nccl|rccl|all_?reduce|step " gpurun_out/dp_trace_${TAG}.txt | head -20
tail -2 gpurun_out/dp_trace_${TAG}.txt
