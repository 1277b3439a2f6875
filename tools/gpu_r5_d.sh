#!/bin/bash
# Round 5: the configs[4] leg's host stall (5-6 s at step ~7): allocator counters, then a HIP runtime trace
set -u
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --dual --base 96 --size 2048 --batch 2 --steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 > gpurun_out/r5d_dual.log 2>&1 || { echo fail1; tail -20 gpurun_out/r5d_dual.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --hip-runtime-trace --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r5d_prof -o r5d -- python3 $GRAFT_REPO_ROOT/bench.py --dual --base 96 --size 2048 --batch 2 --steps 12 --warmup 3 --no-cpu-baseline --dice-size 0 > $GRAFT_REPO_ROOT/gpurun_out/r5d_prof.log 2>&1 || { echo fail2; tail -20 $GRAFT_REPO_ROOT/gpurun_out/r5d_prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(find gpurun_out/r5d_prof -name '*hip_api_trace.csv' | head -1)
python3 - "$f" <<'PY' > gpurun_out/r5d_slow_api.txt
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), r["Function"], r.get("Correlation_Id", "")) for r in rows]
rows.sort(reverse=True)
from collections import Counter
tot = Counter()
for d, f, _ in rows: tot[f] += d
print("slowest calls (ms):")
for d, f, c in rows[:40]: print(f"{d/1e6:10.3f} {f} {c}")
print("total per function (ms):")
for f, d in tot.most_common(25): print(f"{d/1e6:10.3f} {f}")
PY
rm -f $(find gpurun_out/r5d_prof -name '*hip_api_trace.csv') 
echo done
