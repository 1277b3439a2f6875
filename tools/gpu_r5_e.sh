#!/bin/bash
# Round 5: GPU test suite (new tests: fillPoly, pin audits, optimizer state, bench --gpus 2, ragged BN
# stats), then the configs[4] host-stall diagnostics (tools/gpu_r5_d.sh)
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5e_pytest.log 2>&1
rc=$?
tail -5 gpurun_out/r5e_pytest.log
grep -E "pin audit|configs\[1\] logits|ragged offset" gpurun_out/r5e_pytest.log | head -40 > gpurun_out/r5e_audit.txt || true
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_r5_d.sh
