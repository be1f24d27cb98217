set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/t_all.log; exit 1; }
tail -1 gpurun_out/t_all.log
timeout -k 10 900 python -u bench.py > gpurun_out/bench_r2c.json 2> gpurun_out/bench_r2c.err || { echo "bench failed"; tail -20 gpurun_out/bench_r2c.err; exit 1; }
tail -c 600 gpurun_out/bench_r2c.json
