mkdir -p gpurun_out
FBN_PC_TIMING=1 timeout -k 10 200 python -u tools/pc5_timing.py 6 > gpurun_out/pc5a.log 2>&1
