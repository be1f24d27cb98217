set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pc.py -x -v --timeout 120 --timeout-method thread -k "alpha" 2>&1 | tee gpurun_out/t_pc.log | grep -E "PASS|FAIL|ERROR|passed|failed"
