bash tools/gpu_r6c.sh || exit 1
timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6b_ops.log 2>&1; echo "ops rc=$?"; tail -1 gpurun_out/r6b_ops.log
timeout -k 10 700 python -u -m pytest tests/test_gpu_configs.py -x -v -s -k configs2 --timeout 600 --timeout-method thread > gpurun_out/r6b_cfg2.log 2>&1; echo "cfg2 rc=$?"
