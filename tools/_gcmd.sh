mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_jt.py -x -v --timeout 120 --timeout-method thread -k "streamed or synthetic_network or large_batch" > gpurun_out/t4.log 2>&1 && timeout -k 10 600 python -u tools/virt_ablate.py 125000 0,16 > gpurun_out/ablate.log 2>&1
