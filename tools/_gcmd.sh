set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_pc_dist.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_pcd.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/t_pcd.log; exit 1; }
tail -1 gpurun_out/t_pcd.log
timeout -k 10 200 python tools/pc_dist_timing.py 2>&1 | grep -E "median|^pc level|session"
