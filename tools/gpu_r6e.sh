mkdir -p gpurun_out
timeout -k 10 400 python tools/cfg2_loss_probe.py > gpurun_out/r6_lossprobe.txt 2>&1; echo "probe rc=$?"; cat gpurun_out/r6_lossprobe.txt
A="" B="EUNET_LIB=abl/libprev.so" ROUNDS=3 bash tools/gpu_ab_env.sh
