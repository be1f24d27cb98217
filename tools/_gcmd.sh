mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pc.py -x -v --timeout 200 --timeout-method thread -k config5 > gpurun_out/tc5.log 2>&1
