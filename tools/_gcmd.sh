mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pc.py -x -q --timeout 120 --timeout-method thread -k "bit_sliced or synthetic" > gpurun_out/tpc.log 2>&1 && FBN_PC_TIMING=1 timeout -k 10 200 python -u tools/pc5_timing.py 3 > gpurun_out/pc5a.log 2>&1
