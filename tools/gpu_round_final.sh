#!/bin/bash
# Round-end measurement on one GPU: PMC traffic + MFMA passes (their summaries are what bench.py
# reads for roofline.traffic / mfma), a rocprofv3 kernel-trace --stats run of the default bench,
# the default bench itself (CPU baseline + Dice legs) and the fp32 configs[1] line.
set -u
mkdir -p gpurun_out
TAG=${TAG:-final}
TAG=$TAG bash tools/gpu_pmc.sh > gpurun_out/pmc_${TAG}_run.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/pmc_${TAG}_run.log; exit 1; }
TAG=$TAG bash tools/gpu_pmc_mfma.sh > gpurun_out/pmc_${TAG}_mfma_run.log 2>&1 || { echo "pmc mfma failed"; exit 1; }
cp gpurun_out/pmc_${TAG}_summary.json profiles/r02_pmc_summary.json
cp gpurun_out/pmc_${TAG}_mfma_summary.json profiles/r02_pmc_mfma_summary.json
BENCH_ARGS="--steps 10 --warmup 3 --no-cpu-baseline --dice-size 0" TAG=$TAG bash tools/gpu_prof.sh > gpurun_out/prof_${TAG}_run.log 2>&1 || { echo "prof failed"; exit 1; }
timeout -k 10 900 python bench.py > gpurun_out/bench_${TAG}.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench_${TAG}.log; exit 1; }
grep "^{" gpurun_out/bench_${TAG}.log | tail -1 > gpurun_out/bench_${TAG}.json
timeout -k 10 600 python bench.py --base 64 --size 512 --batch 8 --dtype fp32 > gpurun_out/bench_${TAG}_fp32.log 2>&1 || { echo "fp32 bench failed"; exit 1; }
grep "^{" gpurun_out/bench_${TAG}_fp32.log | tail -1 > gpurun_out/bench_${TAG}_fp32.json
echo done
