set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r03s2; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_pc_small.py tests/test_gpu_pc.py -x -q --timeout 120 --timeout-method thread > $o/pcs_t.log 2>&1 || { tail -40 $o/pcs_t.log; exit 1; }
tail -2 $o/pcs_t.log
FBN_PC_SMALL_TRACE=1 timeout -k 10 200 python -u tools/pc_small_timing.py 3 > $o/pcsmall.log 2>&1 || { tail -30 $o/pcsmall.log; exit 1; }
grep "pc small level" $o/pcsmall.log | tail -5
timeout -k 10 200 python -u tools/pc_small_timing.py 200 > $o/pcsmall2.log 2>&1 || { tail -30 $o/pcsmall2.log; exit 1; }
tail -1 $o/pcsmall2.log
