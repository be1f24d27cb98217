# scratch GPU command (gpurun): round-4 session 1 -- changed PC tests + cooperative-launch timing
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r04a; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_pc_small.py tests/test_gpu_gram_mfma.py tests/test_gpu_cli.py tests/test_gpu_pc_dist.py tests/test_gpu_pc_c5_pinned.py -x -v --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || { tail -60 $o/tests.log; exit 1; }
tail -3 $o/tests.log
timeout -k 10 300 python -u tools/pc_small_timing.py 300 > $o/pcsmall.log 2>&1 || { tail -30 $o/pcsmall.log; exit 1; }
cat $o/pcsmall.log | grep -v "^pc small\|^    one-wave"
