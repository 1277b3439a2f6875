# round 6: data-parallel GPU tests incl. the new world-4 mean-of-shards case (4 ranks on the one GPU over gloo)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_dp_gpu.py -v --timeout 600 --timeout-method thread > gpurun_out/r6r_pt.log 2>&1 || { echo "pytest failed"; grep -E "^E |FAILED|Error|passed|failed" gpurun_out/r6r_pt.log | head -30; exit 1; }
grep -E "PASSED|FAILED|mean-of-shards|passed" gpurun_out/r6r_pt.log | head -30
