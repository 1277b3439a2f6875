# the full GPU suite, then the round-6 measurement pass (tools/gpu_r6_final.sh)
set -u
mkdir -p gpurun_out
TAG=full6e TLIM=800 TTIME=600 bash tools/gpu_run_tests.sh tests -m gpu -q || exit 1
grep -q " passed" gpurun_out/pytest_full6e.log && ! grep -q "failed" gpurun_out/pytest_full6e.log || { echo "tests not green"; exit 1; }
TAG=r6i bash tools/gpu_r6_final.sh
