mkdir -p gpurun_out/wt
timeout -k 10 100 python tools/wavetime.py bunny15 256 8 > gpurun_out/wt/wt8.log 2>&1 || exit $?
timeout -k 10 100 python tools/wavetime.py bunny15 32 1 > gpurun_out/wt/wt1.log 2>&1 || exit $?
cat gpurun_out/wt/wt8.log gpurun_out/wt/wt1.log
