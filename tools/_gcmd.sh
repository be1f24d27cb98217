# scratch GPU command (gpurun): round-4 -- tiled kernel: un-normalized messages, direct bin output
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r04t; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_jt_tile.py -x -v --timeout 120 --timeout-method thread > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
tail -2 $o/t.log
timeout -k 10 300 python -u tools/tile_probe.py 125000 6144:16 4096:16 > $o/probe.log 2>&1 || { tail -20 $o/probe.log; exit 1; }
cat $o/probe.log
