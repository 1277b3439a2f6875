#!/bin/bash
# HBM traffic counters of a short bench run: FETCH_SIZE and WRITE_SIZE in SEPARATE
# rocprofv3 passes (they do not fit one TCC pass), kernel-trace only, no sys/runtime trace.
set -u
mkdir -p gpurun_out
TAG=${TAG:-pmc}
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 ${PMC_TIMEOUT:-400} rocprofv3 --pmc $c --kernel-trace --output-format csv \
    -d gpurun_out/pmc_${TAG}_$c -o run -- \
    python bench.py ${BENCH_ARGS:---steps 2 --warmup 1 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg --no-dual-leg} > gpurun_out/pmc_${TAG}_$c.log 2>&1
  rc=$?
  echo "pmc $c rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc_${TAG}_$c.log; exit $rc; fi
done
python tools/pmc_summary.py gpurun_out/pmc_${TAG}_FETCH_SIZE gpurun_out/pmc_${TAG}_WRITE_SIZE ${PMC_WORKLOAD:-64,1024,4,bf16} \
  > gpurun_out/pmc_${TAG}_summary.json
echo "summary rc=$?"; head -c 3000 gpurun_out/pmc_${TAG}_summary.json
