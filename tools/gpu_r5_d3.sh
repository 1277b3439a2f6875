#!/bin/bash
# Round 5: fusion_head.0 on the MFMA forward (DualEngine.narrow_mfma) -- dual parity tests, then alternating bench
# runs with the dual leg (knob on / off)
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dual.py tests/test_gpu_configs.py -x -q -k "dual or configs4 or base96" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5d3_pytest.log 2>&1 || { echo "pytest failed"; grep -E "^E |FAILED|Error" gpurun_out/r5d3_pytest.log | head -20; exit 1; }
tail -1 gpurun_out/r5d3_pytest.log
out=gpurun_out/ab_r5d3.jsonl; : > $out
for r in 1 2 3; do
  for v in base dual.narrow_mfma=0; do
    sets=""; [ $v != base ] && sets=$v
    timeout -k 10 400 python3 tools/ab_attr.py $sets -- --steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg > gpurun_out/ab_r5d3_run.log 2>&1 || { echo "bench failed $v"; tail -5 gpurun_out/ab_r5d3_run.log; exit 1; }
    line=$(grep '^{' gpurun_out/ab_r5d3_run.log | tail -1)
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(json.dumps({'variant': sys.argv[2], 'round': int(sys.argv[3]), 'value': d['value'], 'dual': d['dual_configs4']['value'], 'dual_frac': d['dual_configs4']['roofline']['frac']}))" "$line" "$v" "$r" >> $out
    tail -1 $out
  done
done
