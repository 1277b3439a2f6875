#!/bin/bash
# SQ issue/wait/LDS counters per kernel: one rocprofv3 --pmc pass (8 SQ counters, kernel-trace only).
# PROG: the program (default: a short bench run; e.g. PROG='python tools/head_bench.py --reps 3').
set -u
mkdir -p gpurun_out
TAG=${TAG:-sq}
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
  SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU --kernel-trace --output-format csv -d gpurun_out/pmc_${TAG} -o run -- \
  ${PROG:-python bench.py --steps 2 --warmup 1 --no-cpu-baseline --dice-size 0} > gpurun_out/pmc_${TAG}.log 2>&1
rc=$?; echo "pmc sq rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc_${TAG}.log; exit $rc; fi
python tools/sq_summary.py gpurun_out/pmc_${TAG} > gpurun_out/pmc_${TAG}_summary.txt; echo "summary rc=$?"
cat gpurun_out/pmc_${TAG}_summary.txt
