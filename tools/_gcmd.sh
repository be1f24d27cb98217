# scratch GPU command (gpurun): round-4 -- tiled kernel first run + microbenchmark + changed PC tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r04b; mkdir -p $o
timeout -k 10 120 ./tools/micro/gather_rate > $o/gather_rate.log 2>&1 || { tail -30 $o/gather_rate.log; exit 1; }
cat $o/gather_rate.log
timeout -k 10 300 python -u tools/tile_probe.py 125000 > $o/tile_probe.log 2>&1 || { tail -30 $o/tile_probe.log; exit 1; }
cat $o/tile_probe.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_pc_small.py tests/test_gpu_gram_mfma.py tests/test_gpu_cli.py tests/test_gpu_pc_dist.py tests/test_gpu_pc_c5_pinned.py -x -v --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || { tail -60 $o/tests.log; exit 1; }
tail -3 $o/tests.log
timeout -k 10 300 python -u tools/pc_small_timing.py 300 > $o/pcsmall.log 2>&1 || { tail -30 $o/pcsmall.log; exit 1; }
grep -v "^pc small\|^    one-wave" $o/pcsmall.log
