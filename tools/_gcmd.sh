set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r2b.json 2> gpurun_out/bench_r2b.err || { echo "bench failed"; tail -30 gpurun_out/bench_r2b.err; exit 1; }
echo bench ok
