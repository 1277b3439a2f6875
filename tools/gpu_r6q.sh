# round 6: bf16 data gradient with C^T accumulators (in-tree) vs the C-layout epilogue (abl/libprev.so = 9991742
# conv3x3), step-level repeat with four alternating rounds
mkdir -p gpurun_out
TAG=r6q VARIANTS="base|env:EUNET_LIB=abl/libprev.so" ROUNDS=4 bash tools/gpu_ab_knobs.sh > gpurun_out/r6q_ab.txt 2>&1 || { echo "ab failed"; tail -5 gpurun_out/r6q_ab.txt; exit 1; }
python3 - <<'PY'
import json, collections
v = collections.defaultdict(list)
for l in open("gpurun_out/ab_r6q.jsonl"):
    d = json.loads(l); v[d["variant"]].append(d["value"])
for k, x in v.items(): print(k, x, round(sum(x) / len(x), 2))
PY
