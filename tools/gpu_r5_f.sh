#!/bin/bash
# Round 5: full GPU suite, then the driver's bench command twice (Trainer.max_inflight = 2)
set -u
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5f_pytest.log 2>&1
rc=$?
tail -8 gpurun_out/r5f_pytest.log
grep -E "pin audit|configs\[1\] logits|ragged offset" gpurun_out/r5f_pytest.log > gpurun_out/r5f_audit.txt || true
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 > gpurun_out/r5f_drv$i.log 2>&1 || { echo fail$i; tail -20 gpurun_out/r5f_drv$i.log; exit 1; }
done
echo done
