# round 6: wgrad X-halo DMA coalescing ablation (abl/libwgcoal.so: same bytes pixel-major -- wrong results)
mkdir -p gpurun_out
for L in "" "EUNET_LIB=abl/libwgcoal.so"; do
  for T in "" "--transform"; do
    env $L timeout -k 10 150 python tools/conv_bench.py --reps 10 $T > gpurun_out/r6i_cb.log 2>&1 || { echo cb fail; tail -5 gpurun_out/r6i_cb.log; exit 1; }
    cp gpurun_out/r6i_cb.log "gpurun_out/r6i_cb${L:+_coal}${T:+_t}.jsonl"
    echo "== [$L] [$T] $(grep summary gpurun_out/r6i_cb.log)"
  done
done
