# round 6 end: per-layer SQ attribution of the final conv kernels, plain and with the operand transform
mkdir -p gpurun_out
TAG=r6sqa bash tools/gpu_sq_layers.sh > gpurun_out/r6sqa_run.log 2>&1 || { echo "sq plain failed"; tail -5 gpurun_out/r6sqa_run.log; exit 1; }
TAG=r6sqb PROG="python tools/conv_bench.py --reps 1 --transform" bash tools/gpu_sq_layers.sh > gpurun_out/r6sqb_run.log 2>&1 || { echo "sq transform failed"; tail -5 gpurun_out/r6sqb_run.log; exit 1; }
head -42 gpurun_out/pmc_r6sqa_summary.txt
