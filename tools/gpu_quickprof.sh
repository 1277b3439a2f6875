#!/bin/bash
# Selected GPU tests (TESTS, -k KSEL) then a rocprofv3 kernel-trace --stats bench run; prints the top
# kernels per step.  Stops at the first crash-type exit status.
set -u
mkdir -p gpurun_out
TAG=${TAG:-q}
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest ${TESTS} -m gpu -q -x --timeout 300 --timeout-method thread \
    ${KSEL:+-k "$KSEL"} > gpurun_out/pytest_${TAG}.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_${TAG}.log; grep -E "^FAILED|^E  " gpurun_out/pytest_${TAG}.log | head -5
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
STEPS=${STEPS:-5}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- \
  python bench.py --steps $STEPS --warmup 2 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg ${BENCH_ARGS:-} > gpurun_out/prof_${TAG}.log 2>&1
rc=$?; echo "prof rc=$rc"; grep "^{" gpurun_out/prof_${TAG}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'ms/step', d['ms_per_step'], 'conv frac', d['roofline']['frac'], 'enc', d['roofline'].get('encoder_fwd',{}).get('frac'))"
f=$(find gpurun_out/prof_${TAG} -name '*kernel_stats.csv' | head -1)
python3 tools/kstats.py "$f" $((STEPS + 2)) 18
exit $rc
