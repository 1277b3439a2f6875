# conv A/B over variant libraries: KEY=wgrad_ms bash tools/abl_wg.sh lib1 lib2 ...
for l in "" "$@"; do
  echo "lib=${l:-prod} $(EUNET_LIB=$l timeout -k 10 120 python tools/conv_bench.py --reps 10 --transform | python tools/cb_sum.py ${KEY:-wgrad_ms})"
done
