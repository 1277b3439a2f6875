# round-6 measurement pass: PMC traffic + MFMA (profiles/r06_pmc_*), kernel trace + stats + step timeline,
# DP world-1 trace, SQ per-kernel counters, then the default bench line
set -u
mkdir -p gpurun_out
TAG=${TAG:-r6f} R=r06 bash tools/gpu_round_final.sh || exit 1
TAG=r6sq PROG="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg --no-dual-leg" bash tools/gpu_pmc_sq.sh > gpurun_out/r6sq_run.log 2>&1 || { echo "sq failed"; exit 1; }
cp gpurun_out/pmc_r6sq_summary.txt profiles/r06_sq_kernels.txt
cat gpurun_out/bench_${TAG:-r6f}.json | head -c 1500
