# round 6: ops gates, configs[2] suite, per-layer conv timings with the transform (wgrad remap)
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r6b_ops.log 2>&1; echo "ops rc=$?"
timeout -k 10 200 python tools/conv_bench.py --reps 10 --transform > gpurun_out/cb6b.txt 2>&1; echo "cb rc=$?"
timeout -k 10 700 python -u -m pytest tests/test_gpu_configs.py -x -v -s -k configs2 --timeout 600 --timeout-method thread > gpurun_out/r6b_cfg2.log 2>&1; echo "cfg2 rc=$?"
