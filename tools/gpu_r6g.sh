# round 6: wgrad staging-latency ablation (abl/libwgnost.so: DMA only for a split's first tile -- wrong results,
# timing only), then the full GPU suite
mkdir -p gpurun_out
for L in "" "EUNET_LIB=abl/libwgnost.so"; do
  for T in "" "--transform"; do
    env $L timeout -k 10 150 python tools/conv_bench.py --reps 10 $T > gpurun_out/r6g_cb.log 2>&1 || { echo cb fail; tail -5 gpurun_out/r6g_cb.log; exit 1; }
    cp gpurun_out/r6g_cb.log "gpurun_out/r6g_cb${L:+_nost}${T:+_t}.jsonl"
    echo "== [$L] [$T] $(grep summary gpurun_out/r6g_cb.log)"
  done
done
TAG=full6 TLIM=1000 TTIME=600 bash tools/gpu_run_tests.sh tests -m gpu -q
