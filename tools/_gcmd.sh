set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r02w; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests/test_gpu_pc.py tests/test_gpu_pc_dist.py -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
tail -1 $o/t.log
for v in "FBN_CI_L1G2=0" "FBN_X=0" "FBN_CI_L1G2=0" "FBN_X=0"; do
  echo $v; env $v timeout -k 10 200 python tools/pc5_timing.py 8 2>&1 | grep "run " | tail -1 | sed 's/tests \[.*launched/launched/' || exit 1
done
mkdir -p $o/st
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/st -o run --output-format csv -- python tools/pc5_timing.py 3 > /dev/null 2>&1 || exit 1
