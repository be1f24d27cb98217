set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r03s3; mkdir -p $o
for U in 1 2 1 2; do
  FBN_CI_L1_UNROLL=$U timeout -k 10 200 python -u tools/pc5_timing.py 8 > $o/u_$U.log 2>&1 || { tail -30 $o/u_$U.log; exit 1; }
  echo "U=$U"; tail -3 $o/u_$U.log
done
FBN_CI_L1_UNROLL=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_pc.py tests/test_gpu_pc_c5_pinned.py -x -q --timeout 300 --timeout-method thread > $o/u2_t.log 2>&1 || { tail -40 $o/u2_t.log; exit 1; }
tail -1 $o/u2_t.log
