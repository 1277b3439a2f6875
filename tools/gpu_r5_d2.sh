#!/bin/bash
# Round 5: kernel statistics of the dual-branch configs[4] step (tools/dual_prof.py under rocprofv3)
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r5dual -o run -- python tools/dual_prof.py --steps 3 > gpurun_out/prof_r5dual.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/prof_r5dual.log; exit 1; }
f=$(find gpurun_out/prof_r5dual -name '*kernel_stats.csv' | head -1)
head -30 "$f" | cut -c1-160
