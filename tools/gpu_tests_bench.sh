#!/bin/bash
# Selected GPU tests (TESTS, optional -k KSEL) then the default bench line (BENCH_ARGS appended).
# Each GPU step under its own time limit; stops at the first failure.
set -u
mkdir -p gpurun_out
TAG=${TAG:-tb}
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest ${TESTS} -m gpu -x -v -s --timeout 300 --timeout-method thread \
    ${KSEL:+-k "$KSEL"} > gpurun_out/pytest_${TAG}.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_${TAG}.log | tail -20
  [ $rc -ne 0 ] && { grep -E "^E  " gpurun_out/pytest_${TAG}.log | head -10; exit $rc; }
fi
if [ -z "${NO_BENCH:-}" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-600} python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench_${TAG}.log 2>&1
  rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/bench_${TAG}.log; exit $rc; }
  grep "^{" gpurun_out/bench_${TAG}.log | tail -1 > gpurun_out/bench_${TAG}.json
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${TAG}.json')); r=d['roofline']; print('value', d['value'], 'ms', d['ms_per_step'], 'frac', r['frac'], 'step_frac', r['step_frac'], 'enc', r.get('encoder_fwd',{}).get('frac'), 'dp', d.get('dp_world1'), 'fp32', (d.get('fp32_configs1') or {}).get('value'))"
fi
