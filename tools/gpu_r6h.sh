# round 6: double-buffered weight gradient (in-tree) vs the single-stage one (abl/libprev.so = HEAD conv3x3)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r6h_pt.log 2>&1 || { echo "pytest failed"; grep -E "^E |FAILED|Error" gpurun_out/r6h_pt.log | head -20; exit 1; }
tail -1 gpurun_out/r6h_pt.log
for L in "" "EUNET_LIB=abl/libprev.so"; do
  for T in "" "--transform"; do
    env $L timeout -k 10 150 python tools/conv_bench.py --reps 10 $T > gpurun_out/r6h_cb.log 2>&1 || { echo cb fail; tail -5 gpurun_out/r6h_cb.log; exit 1; }
    cp gpurun_out/r6h_cb.log "gpurun_out/r6h_cb${L:+_prev}${T:+_t}.jsonl"
    echo "== [$L] [$T] $(grep summary gpurun_out/r6h_cb.log)"
  done
done
A="" B="EUNET_LIB=abl/libprev.so" ROUNDS=3 bash tools/gpu_ab_env.sh
