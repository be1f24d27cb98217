mkdir -p gpurun_out
for g in 4 2 3; do for r in 8192 32768; do echo "growth $g round0 $r" >> gpurun_out/grow.log; FBN_PC_GROWTH=$g FBN_PC_ROUND0=$r timeout -k 10 200 python -u tools/pc5_timing.py 3 2>&1 | grep "^run 2" >> gpurun_out/grow.log || exit 1; done; done
