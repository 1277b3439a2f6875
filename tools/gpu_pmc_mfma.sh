#!/bin/bash
# MFMA-pipe utilisation + effective clock per kernel: one rocprofv3 --pmc pass (kernel-trace only).
set -u
mkdir -p gpurun_out
TAG=${TAG:-mfma}
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 ${PMC_TIMEOUT:-400} rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
  -d gpurun_out/pmc_${TAG}_mfma -o run -- \
  python bench.py ${BENCH_ARGS:---steps 2 --warmup 1 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg --no-dual-leg} > gpurun_out/pmc_${TAG}_mfma.log 2>&1
rc=$?
echo "pmc mfma rc=$rc"
if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc_${TAG}_mfma.log; exit $rc; fi
python tools/mfma_summary.py gpurun_out/pmc_${TAG}_mfma > gpurun_out/pmc_${TAG}_mfma_summary.json
echo "summary rc=$?"; head -c 2500 gpurun_out/pmc_${TAG}_mfma_summary.json
