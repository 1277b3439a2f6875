# round 6: weight-gradient X halo in octant-pair planes (in-tree) vs octant planes (abl/libprev.so = HEAD)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_dual.py -x -q --timeout 300 --timeout-method thread -k "wgrad or conv3x3 or bf16 or exact or grads or per_sample" > gpurun_out/r6l_pt.log 2>&1 || { echo "pytest failed"; grep -E "^E |FAILED|Error" gpurun_out/r6l_pt.log | head -20; exit 1; }
tail -1 gpurun_out/r6l_pt.log
for L in "" "EUNET_LIB=abl/libprev.so"; do
  for T in "" "--transform"; do
    env $L timeout -k 10 150 python tools/conv_bench.py --reps 10 $T > gpurun_out/r6l_cb.log 2>&1 || { echo cb fail; tail -5 gpurun_out/r6l_cb.log; exit 1; }
    cp gpurun_out/r6l_cb.log "gpurun_out/r6l_cb${L:+_prev}${T:+_t}.jsonl"
    echo "== [$L] [$T] $(grep summary gpurun_out/r6l_cb.log)"
  done
done
TAG=r6l VARIANTS="base|env:EUNET_LIB=abl/libprev.so" ROUNDS=3 bash tools/gpu_ab_knobs.sh > gpurun_out/r6l_ab.txt 2>&1
python3 - <<'PY'
import json, collections
v = collections.defaultdict(list)
for l in open("gpurun_out/ab_r6l.jsonl"):
    d = json.loads(l); v[d["variant"]].append(d["value"])
for k, x in v.items(): print(k, x, round(sum(x) / len(x), 2))
PY
