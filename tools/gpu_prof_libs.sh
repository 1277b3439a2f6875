#!/bin/bash
# rocprofv3 --kernel-trace --stats of the bench workload for each library in LIBS (tools/ab_attr.py
# with ATTRS), then a per-kernel ms/step comparison (tools/cmp_kstats.py).
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
dirs=""
for L in $LIBS; do
  t=$(basename $L .so)
  timeout -k 10 300 env EUNET_LIB=$L rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profl_$t -o run -- \
    python tools/ab_attr.py ${ATTRS:-} -- --steps 8 --warmup 3 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg \
    > gpurun_out/profl_$t.log 2>&1 || { echo "prof failed $L"; tail -3 gpurun_out/profl_$t.log; exit 1; }
  grep "^{" gpurun_out/profl_$t.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', d['value'], d['ms_per_step'])"
  dirs="$dirs gpurun_out/profl_$t/run_kernel_stats.csv"
done
python3 tools/cmp_kstats.py 11 $dirs
