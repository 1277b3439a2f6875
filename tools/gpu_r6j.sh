# round 6: wave-local wgrad transform (no block barrier) vs abl/libprev.so (HEAD), plus pool_recompute
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread -k "wgrad or conv3x3 or bf16 or exact or grads" > gpurun_out/r6j_pt.log 2>&1 || { echo "pytest failed"; grep -E "^E |FAILED|Error" gpurun_out/r6j_pt.log | head -20; exit 1; }
tail -1 gpurun_out/r6j_pt.log
for L in "" "EUNET_LIB=abl/libprev.so"; do
  env $L timeout -k 10 150 python tools/conv_bench.py --reps 10 --transform > gpurun_out/r6j_cb.log 2>&1 || { echo cb fail; tail -5 gpurun_out/r6j_cb.log; exit 1; }
  cp gpurun_out/r6j_cb.log "gpurun_out/r6j_cb${L:+_prev}.jsonl"
  echo "== [$L] $(grep summary gpurun_out/r6j_cb.log)"
done
TAG=r6j VARIANTS="base|env:EUNET_LIB=abl/libprev.so|pool_recompute=1" ROUNDS=3 bash tools/gpu_ab_knobs.sh > gpurun_out/r6j_ab.txt 2>&1
python3 - <<'PY'
import json, collections
v = collections.defaultdict(list)
for l in open("gpurun_out/ab_r6j.jsonl"):
    d = json.loads(l); v[d["variant"]].append(d["value"])
for k, x in v.items(): print(k, x, round(sum(x) / len(x), 2))
PY
