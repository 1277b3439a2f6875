#!/bin/bash
# bench A/B of runtime variants: CONFIGS="A=1 B=2;C=0;..." (each item = env assignments, "X=0" = default)
set -u
mkdir -p gpurun_out
TAG=${TAG:-ab}
IFS=';' read -ra CF <<< "${CONFIGS:-X=0}"
for rep in $(seq ${REPS:-2}); do
  for v in "${CF[@]}"; do
    env $v timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --dice-size 0 ${BENCH_ARGS:-} \
      > gpurun_out/bench_${TAG}.log 2>&1
    rc=$?; if [ $rc -ne 0 ]; then echo "bench rc=$rc ($v)"; tail -5 gpurun_out/bench_${TAG}.log; exit $rc; fi
    python -c "import json; d=json.loads(open('gpurun_out/bench_${TAG}.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$v'.ljust(48), d['value'], d['ms_per_step'], r['kernel_ms_per_step'], r.get('wgrad_ms_per_step'))"
  done
done
