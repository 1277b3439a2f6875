#!/bin/bash
# Persistent Cin=64 conv kernel: GPU conv tests, its ablation, per-layer timing with it on and off.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -q -k "conv3x3" --timeout 200 --timeout-method thread > gpurun_out/pytest_k64.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 gpurun_out/pytest_k64.log)"; if [ $rc -ne 0 ]; then grep -E "^FAILED|^E  " gpurun_out/pytest_k64.log | head; exit $rc; fi
ABLATE_K64=1 timeout -k 10 120 tools/conv_ablate 4 1024 1024 64 64 10 && ABLATE_ISC=1 ABLATE_K64=1 timeout -k 10 120 tools/conv_ablate 4 1024 1024 64 64 10 || exit 1
for v in 1 0; do
  for l in ${LAYERS:-enc1.3 enc2.0 dec2.0 dec2.3}; do
    EUNET_CONV_K64=$v timeout -k 10 120 python tools/conv_bench.py --only $l --reps 10 2>/dev/null | grep layer | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('k64=$v', d['layer'], d['fwd_ms'], d['fwd_tf'], d['dgrad_ms'], d['dgrad_tf'])" || exit 1
  done
done
