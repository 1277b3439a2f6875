# round 6: conv layout A/B (in-tree: half-plane DMA halo + wgrad transform remap; B: abl/libprev.so = round 5)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread -k "conv" > gpurun_out/r6c_ops.log 2>&1 || { echo "ops failed"; grep -E "^E |FAILED|Error" gpurun_out/r6c_ops.log | head -20; exit 1; }
tail -1 gpurun_out/r6c_ops.log
for L in "" "EUNET_LIB=abl/libprev.so"; do
  for T in "" "--transform"; do
    env $L timeout -k 10 150 python tools/conv_bench.py --reps 10 $T > gpurun_out/r6c_cb.log 2>&1 || { echo cb fail; tail -5 gpurun_out/r6c_cb.log; exit 1; }
    cp gpurun_out/r6c_cb.log "gpurun_out/r6c_cb_${L:+prev}${T:+_t}.jsonl"
    echo "== [$L] [$T] $(grep summary gpurun_out/r6c_cb.log)"
  done
done
A="" B="EUNET_LIB=abl/libprev.so" ROUNDS=${ROUNDS:-2} bash tools/gpu_ab_env.sh
