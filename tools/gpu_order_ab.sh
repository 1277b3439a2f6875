#!/bin/bash
# A/B of the conv block orders in the full bench (EUNET_CONV_ORDER / EUNET_WGRAD_ORDER)
set -u
mkdir -p gpurun_out
TAG=${TAG:-order}
for cfg in "0 0" "1 0" "2 0" "1 1" "0 1" "0 0" "1 0"; do
  set -- $cfg
  EUNET_CONV_ORDER=$1 EUNET_WGRAD_ORDER=$2 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline \
    --dice-size 0 > gpurun_out/bench_${TAG}_$1$2.log 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "bench rc=$rc ($cfg)"; tail -5 gpurun_out/bench_${TAG}_$1$2.log; exit $rc; fi
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_${TAG}_$1$2.log').read().strip().splitlines()[-1]); print('conv_order=$1 wgrad_order=$2', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_step'], d['roofline']['wgrad_ms_per_step'])"
done
