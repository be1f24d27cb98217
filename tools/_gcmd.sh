mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_jt.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t4.log 2>&1
