mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_all.log 2>&1 && FBN_PC_TIMING=1 timeout -k 10 200 python -u tools/pc5_timing.py 5 > gpurun_out/pc5a.log 2>&1 && timeout -k 10 100 python -u tools/pc_alarm_levels.py 5 > gpurun_out/pal0.log 2>&1
