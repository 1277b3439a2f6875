#!/bin/bash
# SQ counters on one conv layer (tools/conv_bench.py --only LAYER): one rocprofv3 --pmc pass.
set -u
mkdir -p gpurun_out
L=${1:-dec2.3}; TAG=${TAG:-convsq}
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
  SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU --kernel-trace --output-format csv -d gpurun_out/pmc_${TAG} -o run -- \
  python tools/conv_bench.py --only $L --reps 3 --transform > gpurun_out/pmc_${TAG}.log 2>&1
rc=$?; echo "pmc rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc_${TAG}.log; exit $rc; fi
python tools/sq_summary.py gpurun_out/pmc_${TAG}
