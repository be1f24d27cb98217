set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_jt.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_jt.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/t_jt.log; exit 1; }
tail -1 gpurun_out/t_jt.log
for v in "" "FBN_JT_VDEBUG=1024"; do
echo "== $v"; env $v timeout -k 10 200 python tools/munin_once.py 125000 2>&1 | tail -1
env $v timeout -k 10 200 python tools/munin_once.py 125000 2>&1 | tail -1
done
