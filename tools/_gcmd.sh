set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r03s3; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_pc.py tests/test_gpu_pc_c5_pinned.py -x -q --timeout 300 --timeout-method thread > $o/w_t.log 2>&1 || { tail -40 $o/w_t.log; exit 1; }
tail -1 $o/w_t.log
for r in 1 2; do
  timeout -k 10 200 python -u tools/pc5_timing.py 8 > $o/w_$r.log 2>&1 || { tail -30 $o/w_$r.log; exit 1; }
  FBN_PC_TIMING=1 timeout -k 10 200 python -u tools/pc5_timing.py 6 > $o/wt_$r.log 2>&1 || { tail -30 $o/wt_$r.log; exit 1; }
  tail -2 $o/w_$r.log; grep "pc level 1:" $o/wt_$r.log | tail -3
done
