set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_pc.py tests/test_gpu_pc_dist.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_pc.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/t_pc.log; exit 1; }
tail -1 gpurun_out/t_pc.log
echo "default"; timeout -k 10 120 python tools/pc5_timing.py 5 2>&1 | grep -E "run " | tail -1
timeout -k 10 120 python tools/pc_alarm_timing.py 2>&1 | tail -1
