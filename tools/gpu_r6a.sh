set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_loss_api.py tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread -k "bad_target or out_of_range or trainer_step or step_graph" > gpurun_out/r6a_pytest.log 2>&1; echo "pytest rc=$?"
TAG=sql6 bash tools/gpu_sq_layers.sh > gpurun_out/sql6.txt 2>&1 && TAG=sql6t PROG="python tools/conv_bench.py --reps 1 --transform" bash tools/gpu_sq_layers.sh > gpurun_out/sql6t.txt 2>&1 && timeout -k 10 200 python tools/conv_bench.py --reps 10 --transform > gpurun_out/cb6.txt 2>&1
