#!/bin/bash
# Per-layer SQ stall attribution of the conv3x3 kernels (fwd / dgrad / wgrad of the 13 cfg3 layers):
# three rocprofv3 --pmc passes (8 SQ counters at most each, kernel-trace only) over tools/conv_bench.py,
# joined per dispatch by tools/sq_layers.py.
set -u
mkdir -p gpurun_out
TAG=${TAG:-sql}
PROG=${PROG:-python tools/conv_bench.py --reps 1}
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i + 1))
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/pmc_${TAG}_$i -o run -- \
    $PROG > gpurun_out/pmc_${TAG}_$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc_${TAG}_$i.log; exit $rc; fi
done
SQ_BY_KERNEL=${SQ_BY_KERNEL:-0} python tools/sq_layers.py gpurun_out/pmc_${TAG}_1 gpurun_out/pmc_${TAG}_2 > gpurun_out/pmc_${TAG}_summary.txt
echo "summary rc=$?"
cat gpurun_out/pmc_${TAG}_summary.txt
