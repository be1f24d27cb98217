set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r02m; mkdir -p $o
FBN_PC_TIMING=1 timeout -k 10 200 python tools/pc5_timing.py 3 > $o/pc5_levels.log 2>&1 || { tail $o/pc5_levels.log; exit 1; }
grep "orient:" $o/pc5_levels.log | tail -1
timeout -k 10 200 python tools/pc5_timing.py 8 2>&1 | grep "run " | tail -2 | sed 's/tests \[.*launched/launched/' || exit 1
timeout -k 10 120 python tools/pc_alarm_cabi.py 300 "alarm" 2>&1 | tail -1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_pc.py tests/test_gpu_pc_dist.py tests/test_gpu_cli.py -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
tail -1 $o/t.log
