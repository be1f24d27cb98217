set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r03s3; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_pc.py tests/test_gpu_pc_c5_pinned.py -x -q --timeout 300 --timeout-method thread > $o/p_t.log 2>&1 || { tail -40 $o/p_t.log; exit 1; }
tail -1 $o/p_t.log
for P in 0 1 0 1; do
  FBN_CI_L1_PAIRED=$P timeout -k 10 200 python -u tools/pc5_timing.py 8 > $o/p_$P.log 2>&1 || { tail -30 $o/p_$P.log; exit 1; }
  FBN_PC_TIMING=1 FBN_CI_L1_PAIRED=$P timeout -k 10 200 python -u tools/pc5_timing.py 6 > $o/pt_$P.log 2>&1 || { tail -30 $o/pt_$P.log; exit 1; }
  echo "P=$P"; tail -2 $o/p_$P.log; grep "pc level 1:" $o/pt_$P.log | tail -3
done
