mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pc.py tests/test_gpu_pc_dist.py tests/test_gpu_cli.py -x -q --timeout 200 --timeout-method thread > gpurun_out/tpc.log 2>&1 && FBN_PC_TIMING=1 timeout -k 10 200 python -u tools/pc5_timing.py 3 > gpurun_out/pc5a.log 2>&1
