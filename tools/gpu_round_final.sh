#!/bin/bash
# Round-end measurement on one GPU: PMC traffic + MFMA passes (their summaries are what bench.py
# reads for roofline.traffic / components), a rocprofv3 kernel-trace --stats run of the default bench's
# timed workload, the DataParallel trace, then the default bench line itself (CPU baseline, DP and fp32
# legs, Dice).  R names the round's profile files (profiles/${R}_*).
set -u
mkdir -p gpurun_out
TAG=${TAG:-final}
R=${R:-r03}
TAG=$TAG bash tools/gpu_pmc.sh > gpurun_out/pmc_${TAG}_run.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/pmc_${TAG}_run.log; exit 1; }
TAG=$TAG bash tools/gpu_pmc_mfma.sh > gpurun_out/pmc_${TAG}_mfma_run.log 2>&1 || { echo "pmc mfma failed"; exit 1; }
cp gpurun_out/pmc_${TAG}_summary.json profiles/${R}_pmc_summary.json
cp gpurun_out/pmc_${TAG}_mfma_summary.json profiles/${R}_pmc_mfma_summary.json
BENCH_ARGS="--steps 10 --warmup 3 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg --no-dual-leg" TAG=$TAG bash tools/gpu_prof.sh > gpurun_out/prof_${TAG}_run.log 2>&1 || { echo "prof failed"; exit 1; }
f=$(find gpurun_out/prof_${TAG} -name '*kernel_stats.csv' | head -1); cp "$f" profiles/${R}_bench_kernel_stats.csv
f=$(find gpurun_out/prof_${TAG} -name '*kernel_trace.csv' | head -1)
python3 tools/trace_steps.py "$f" 3 40 > profiles/${R}_step_timeline.txt
TAG=${TAG}dp bash tools/gpu_dp_trace.sh > gpurun_out/dp_${TAG}_run.log 2>&1 || { echo "dp trace failed"; exit 1; }
cp gpurun_out/dp_trace_${TAG}dp.txt profiles/${R}_dp_world1_timeline.txt
timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_${TAG}.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench_${TAG}.log; exit 1; }
grep "^{" gpurun_out/bench_${TAG}.log | tail -1 > gpurun_out/bench_${TAG}.json
cp gpurun_out/bench_${TAG}.json profiles/${R}_bench.json
echo done
