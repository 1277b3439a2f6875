#!/bin/bash
# Same-box A/B of UNetEngine knob settings on the default bench workload, alternating rounds.
#   VARIANTS="base|fuse_bn_apply={enc4,dec4}|arg:--step-graph 1" ROUNDS=3 bash tools/gpu_ab_knobs.sh
# ("base" = no override, "arg:..." = extra bench arguments); one JSON line per run in gpurun_out/ab_<tag>.jsonl
set -u
mkdir -p gpurun_out
TAG=${TAG:-knobs}
ROUNDS=${ROUNDS:-3}
ARGS=${ARGS:-"--steps 30 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg --no-dual-leg"}
IFS='|' read -ra VS <<< "${VARIANTS:-base}"
out=gpurun_out/ab_${TAG}.jsonl
: > $out
for r in $(seq 1 $ROUNDS); do
  for v in "${VS[@]}"; do
    sets=""; extra=""; envs=""
    case "$v" in
      base) ;;
      arg:*) extra="${v#arg:}" ;;   # bench arguments, e.g. arg:--step-graph 1
      env:*) envs="${v#env:}" ;;    # environment, e.g. env:EUNET_LIB=abl/libwg1.so (an A/B build)
      *) sets="$v" ;;
    esac
    env $envs timeout -k 10 200 python3 tools/ab_attr.py $sets -- $ARGS $extra > gpurun_out/ab_${TAG}_run.log 2>&1 || { echo "fail: $v"; tail -20 gpurun_out/ab_${TAG}_run.log; exit 1; }
    line=$(grep '^{' gpurun_out/ab_${TAG}_run.log | tail -1)
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(json.dumps({'variant': sys.argv[2], 'round': int(sys.argv[3]), 'value': d['value'], 'ms': d['ms_per_step'], 'step_ms': d['steps_diag']['step_ms'], 'busy': d['steps_diag']['step_kernel_busy_ms']}))" "$line" "$v" "$r" >> $out
    tail -1 $out
  done
done
echo done
