#!/bin/bash
# Alternating same-box A/B of two configurations, ROUNDS pairs.  A / B: "name=0/1 ..." UNetEngine
# attributes; AENV / BENV: environment assignments for that side (e.g. BENV="EUNET_LIB=abl/lib_r2.so").
set -u
mkdir -p gpurun_out
for i in $(seq 1 ${ROUNDS:-3}); do
  for tag in A B; do
    sets=${!tag}
    envv=${tag}ENV
    timeout -k 10 200 env ${!envv:-} python tools/ab_attr.py $sets -- --steps 30 --warmup 5 --no-cpu-baseline --dice-size 0 \
      --no-dp-world1 --no-fp32-leg > gpurun_out/ab_attr.log 2>&1 || { echo "bench failed ($sets)"; tail -3 gpurun_out/ab_attr.log; exit 1; }
    grep "^{" gpurun_out/ab_attr.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag [$sets ${!envv:-}]', d['value'], d['ms_per_step'])"
  done
done
