mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pc.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tpc.log 2>&1
