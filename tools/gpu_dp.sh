#!/bin/bash
# DP rehearsal on one GPU: the gpu DP test, then a 2-rank bench over gloo (both ranks on cuda:0)
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_dp_gpu.py -q --timeout 500 > gpurun_out/pytest_dp.log 2>&1
rc=$?; echo "dp test rc=$rc"; tail -5 gpurun_out/pytest_dp.log
if [ $rc -ne 0 ]; then exit $rc; fi
EUNET_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/bench_dp2.log 2>&1
rc=$?; echo "bench dp2 rc=$rc"; tail -3 gpurun_out/bench_dp2.log
exit $rc
