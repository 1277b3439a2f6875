set -u
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_eval.py tests/test_gpu_loss_api.py tests/test_gpu_imgproc.py tests/test_gpu_dual.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/t1.log 2>&1
echo "rc=$?"; grep -E "passed|failed|^FAILED|^ERROR" gpurun_out/t1.log | tail -30
