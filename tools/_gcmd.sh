# scratch GPU command (gpurun): round-4 -- 4-wave tiled kernel + in-kernel level-1 offset scan
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r04w; mkdir -p $o
FBN_JT_NO_FIXUP=1 timeout -k 10 120 python -u tools/tile_dbg.py > $o/dbg.log 2>&1 || { tail -20 $o/dbg.log; exit 1; }
cat $o/dbg.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_jt_tile.py tests/test_gpu_jt_fast.py tests/test_gpu_pc.py tests/test_gpu_pc_c5_pinned.py tests/test_gpu_pc_dist.py -x -v --timeout 200 --timeout-method thread > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
tail -2 $o/t.log
timeout -k 10 200 python -u tools/pc5_timing.py 5 > $o/pc5.log 2>&1 || { tail -20 $o/pc5.log; exit 1; }
cat $o/pc5.log
timeout -k 10 400 python -u tools/tile_probe.py 125000 24576:16 16384:16 30720:16 > $o/probe.log 2>&1 || { tail -20 $o/probe.log; exit 1; }
cat $o/probe.log
