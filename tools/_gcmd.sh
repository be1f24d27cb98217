mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_jt.py tests/test_gpu_cli.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tjt.log 2>&1 && timeout -k 10 300 python -u bench.py --steps 10 --no-pc --no-munin --no-baseline > gpurun_out/b1.json 2> gpurun_out/b1.err
