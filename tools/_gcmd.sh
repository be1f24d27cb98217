mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pc.py tests/test_gpu_pc_dist.py tests/test_gpu_cli.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tpc.log 2>&1 && timeout -k 10 100 python -u tools/pc_alarm_levels.py 5 > gpurun_out/pal0.log 2>&1
