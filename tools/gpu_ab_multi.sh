#!/bin/bash
# Alternating same-box comparison of several configurations, ROUNDS rounds.  CFGS: ';'-separated
# entries "label|ENV=... ...|attr=0/1 ..." (ENV part: environment assignments, e.g. EUNET_LIB=abl/x.so;
# attr part: UNetEngine attributes for tools/ab_attr.py).
set -u
mkdir -p gpurun_out
IFS=';' read -ra C <<< "$CFGS"
for i in $(seq 1 ${ROUNDS:-2}); do
  for c in "${C[@]}"; do
    IFS='|' read -r label envs sets <<< "$c"
    timeout -k 10 200 env $envs python tools/ab_attr.py $sets -- --steps 30 --warmup 5 --no-cpu-baseline --dice-size 0 \
      --no-dp-world1 --no-fp32-leg > gpurun_out/ab_multi.log 2>&1 || { echo "bench failed ($label)"; tail -3 gpurun_out/ab_multi.log; exit 1; }
    grep "^{" gpurun_out/ab_multi.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$label', d['value'], d['ms_per_step'])"
  done
done
