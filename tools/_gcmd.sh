# scratch GPU command (gpurun): config-5 orientation timing + PC tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r03s3; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_pc.py tests/test_gpu_cli.py -x -q --timeout 300 --timeout-method thread > $o/o_t.log 2>&1 || { tail -40 $o/o_t.log; exit 1; }
tail -1 $o/o_t.log
timeout -k 10 200 python -u tools/pc5_timing.py 8 > $o/o_1.log 2>&1 || { tail -30 $o/o_1.log; exit 1; }
FBN_PC_TIMING=1 timeout -k 10 200 python -u tools/pc5_timing.py 6 > $o/ot_1.log 2>&1 || { tail -30 $o/ot_1.log; exit 1; }
tail -2 $o/o_1.log; grep "orient:\|pc_stable:" $o/ot_1.log | tail -4
