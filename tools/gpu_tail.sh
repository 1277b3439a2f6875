#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_dual.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/pytest_tail.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 gpurun_out/pytest_tail.log)"; if [ $rc -ne 0 ]; then grep -E "^FAILED|^E  " gpurun_out/pytest_tail.log | head; exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --dice-size 0 > gpurun_out/bench_tail.log 2>&1 || exit $?
tail -1 gpurun_out/bench_tail.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg3', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_step'], d['roofline']['wgrad_ms_per_step'])"
timeout -k 10 600 python bench.py --dual --base 96 --size 2048 --batch 2 --steps 3 --warmup 1 --no-cpu-baseline --dice-size 0 > gpurun_out/bench_dual_tail.log 2>&1 || exit $?
tail -1 gpurun_out/bench_dual_tail.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg5', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_step'], d['roofline']['wgrad_ms_per_step'], d['model_tflops_per_gpu'])"
