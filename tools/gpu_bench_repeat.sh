# smoke() and the default bench command N times back to back on one box (run-to-run spread for the README)
mkdir -p gpurun_out
TAG=${TAG:-rep}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
: > gpurun_out/${TAG}_bench.jsonl
for i in $(seq 1 ${N:-3}); do
  timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_$i.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/${TAG}_bench_$i.log; exit 1; }
  grep "^{" gpurun_out/${TAG}_bench_$i.log | tail -1 >> gpurun_out/${TAG}_bench.jsonl
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['components']['dgrad']['clock_ghz'] if 'clock_ghz' in d['roofline']['components']['dgrad'] else '')" gpurun_out/${TAG}_bench.jsonl $i
done
