set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r02f; mkdir -p $o
timeout -k 10 120 python tools/pc_alarm_cabi.py 200 "orient-vec" 2>&1 | tail -1 || exit 1
FBN_PC_TIMING=1 timeout -k 10 120 python tools/pc_alarm_levels.py 3 > $o/levels.log 2>&1 || exit 1
grep -E "orient|pc_stable:" $o/levels.log | tail -2
timeout -k 10 600 python -u -m pytest tests/test_gpu_pc.py tests/test_gpu_pc_dist.py tests/test_gpu_cli.py -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
tail -1 $o/t.log
