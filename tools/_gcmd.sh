timeout -k 10 300 python -u -m pytest tests/test_gpu_pc.py tests/test_gpu_pc_dist.py tests/test_gpu_cli.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tpc.log 2>&1 && timeout -k 10 120 python -u tools/pc_alarm_timing.py > gpurun_out/pca.log 2>&1 && FBN_PC_TIMING=1 timeout -k 10 120 python -u -c "
import sys; sys.path.insert(0,'.')
import fastbn_amd as F
ds = F.Dataset('tests/golden/alarm/alarm_s5000.txt'); ci = F.IndependenceTest(ds); pc = F.PCStable(0.05, 1000)
for _ in range(4): pc.StructLearnCompData(ci)
" > gpurun_out/pca2.log 2>&1
