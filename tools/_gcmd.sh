mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_all.log 2>&1 && FBN_PC_TIMING=1 timeout -k 10 200 python -u tools/pc5_timing.py 3 > gpurun_out/pc5a.log 2>&1
