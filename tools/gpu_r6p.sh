# round 6: transformed forward (bf16) accumulating C^T (conv3x3, vs abl/libprev.so = HEAD conv3x3) and head_gh at
# 4 waves / SIMD with a one-row W1-gradient tile (vs abl/libhprev.so = HEAD head.hip)
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_dual.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6p_pt.log 2>&1 || { echo "pytest failed"; grep -E "^E |FAILED|Error" gpurun_out/r6p_pt.log | head -20; exit 1; }
tail -1 gpurun_out/r6p_pt.log
LIBS="abl/libhprev.so" TAG=r6p bash tools/gpu_head_libs.sh > gpurun_out/r6p_head.log 2>&1 || { echo "head libs failed"; tail -5 gpurun_out/r6p_head.log; exit 1; }
cat gpurun_out/r6p_head.log
for L in "" "EUNET_LIB=abl/libprev.so"; do
  for T in "" "--transform"; do
    env $L timeout -k 10 150 python tools/conv_bench.py --reps 10 $T > gpurun_out/r6p_cb.log 2>&1 || { echo cb fail; tail -5 gpurun_out/r6p_cb.log; exit 1; }
    cp gpurun_out/r6p_cb.log "gpurun_out/r6p_cb${L:+_prev}${T:+_t}.jsonl"
    echo "== [$L] [$T] $(grep summary gpurun_out/r6p_cb.log)"
  done
done
TAG=r6p VARIANTS="base|env:EUNET_LIB=abl/libprev.so|env:EUNET_LIB=abl/libhprev.so" ROUNDS=3 bash tools/gpu_ab_knobs.sh > gpurun_out/r6p_ab.txt 2>&1
python3 - <<'PY'
import json, collections
v = collections.defaultdict(list)
for l in open("gpurun_out/ab_r6p.jsonl"):
    d = json.loads(l); v[d["variant"]].append(d["value"])
for k, x in v.items(): print(k, x, round(sum(x) / len(x), 2))
PY
