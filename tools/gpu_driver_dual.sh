#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_driver.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_driver.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|SKIPPED|^E  " gpurun_out/pytest_driver.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --dual --base 96 --size 2048 --batch 2 --steps 3 --warmup 1 --no-cpu-baseline --dice-size 0 > gpurun_out/bench_dual_cfg5.log 2>&1
brc=$?; echo "dual bench rc=$brc"; tail -2 gpurun_out/bench_dual_cfg5.log | cut -c1-1500
exit $brc
