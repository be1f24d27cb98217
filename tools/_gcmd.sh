set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r03s2; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_pc_small.py -x -q --timeout 120 --timeout-method thread > $o/pcs_t.log 2>&1 || { tail -40 $o/pcs_t.log; exit 1; }
tail -1 $o/pcs_t.log
for K in 8 4 6 12 16 8; do
  FBN_PC_SPEC_A=$K timeout -k 10 200 python -u tools/pc_small_timing.py 200 > $o/spec_$K.log 2>&1 || { tail -30 $o/spec_$K.log; exit 1; }
  echo "K=$K $(tail -1 $o/spec_$K.log)"
done
