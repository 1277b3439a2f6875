set -e
mkdir -p gpurun_out
: > gpurun_out/abl.txt
for lib in "" $ABL_LIBS; do
  for L in ${ABL_LAYERS:-dec2.3 enc2.0}; do
    echo "lib=${lib:-prod} $(EUNET_LIB=$lib timeout -k 10 60 python tools/conv_bench.py --reps 20 --transform --only $L | grep fwd_ms)" >> gpurun_out/abl.txt
  done
done
