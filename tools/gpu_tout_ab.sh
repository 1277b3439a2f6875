#!/bin/bash
# correctness of a runtime kernel variant (VAR=NAME=VALUE) on the GPU tests, then bench A/B vs default
set -u
mkdir -p gpurun_out
TAG=${TAG:-var}
VAR=${VAR:-EUNET_CONV_TOUT=1}
env $VAR timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_dual.py} -m gpu -q \
  --timeout 200 --timeout-method thread -x > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?; echo "pytest ($VAR) rc=$rc"; tail -4 gpurun_out/pytest_${TAG}.log
if [ $rc -ne 0 ]; then grep -E "^E " gpurun_out/pytest_${TAG}.log | head -20; exit $rc; fi
for v in "X=0" "$VAR" "X=0" "$VAR"; do
  env $v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --dice-size 0 > gpurun_out/bench_${TAG}.log 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "bench rc=$rc ($v)"; tail -5 gpurun_out/bench_${TAG}.log; exit $rc; fi
  python -c "import json; d=json.loads(open('gpurun_out/bench_${TAG}.log').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_step'], d['roofline']['wgrad_ms_per_step'])"
done
