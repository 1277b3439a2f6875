#!/bin/bash
set -u
TAG=pins TLIM=600 bash tools/gpu_run_tests.sh tests/test_gpu_model.py -k "train_grads_match_oracle or multitile" || exit $?
TAG=pinsd TLIM=600 bash tools/gpu_run_tests.sh tests/test_gpu_dual.py -k "train_grads" || exit $?
TAG=cfgs TLIM=700 bash tools/gpu_run_tests.sh tests/test_gpu_configs.py || exit $?
TAG=dp2 TLIM=700 bash tools/gpu_run_tests.sh tests/test_dp_gpu.py -k "trainer_steps or mean_of_shards" || exit $?
bash tools/gpu_r4_sq.sh
