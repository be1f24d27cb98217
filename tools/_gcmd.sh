mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_all.log 2>&1 && timeout -k 10 300 python -u bench.py > gpurun_out/b1.json 2> gpurun_out/b1.err
