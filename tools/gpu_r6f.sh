# round 6: configs[2] loss / slice tests, optimizer test, single-round-trip chunk staging A/B (abl/libstage1.so)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_optim.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6f_optim.log 2>&1; echo "optim rc=$?"; tail -1 gpurun_out/r6f_optim.log
timeout -k 10 700 python -u -m pytest tests/test_gpu_configs.py -x -v -s -k "configs2_loss or configs2_256" --timeout 600 --timeout-method thread > gpurun_out/r6f_cfg2.log 2>&1; echo "cfg2 rc=$?"; grep -E "PASSED|FAILED|configs\[2\]" gpurun_out/r6f_cfg2.log | head
for L in "" "EUNET_LIB=abl/libstage1.so"; do
  env $L timeout -k 10 150 python tools/conv_bench.py --reps 10 --transform > gpurun_out/r6f_cb.log 2>&1 || { echo cb fail; tail -5 gpurun_out/r6f_cb.log; exit 1; }
  cp gpurun_out/r6f_cb.log "gpurun_out/r6f_cb${L:+_stage1}.jsonl"
  echo "== [$L] $(grep summary gpurun_out/r6f_cb.log)"
done
A="" B="EUNET_LIB=abl/libstage1.so" ROUNDS=3 bash tools/gpu_ab_env.sh
