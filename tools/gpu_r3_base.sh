set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3_base_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r3_base_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 > gpurun_out/r3_base_bench.log 2>&1 || exit 1
grep "^{" gpurun_out/r3_base_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'ms/step', d['ms_per_step'])"
