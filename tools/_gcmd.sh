# scratch GPU command (gpurun): round-4 -- tiled kernel with the LRU-aware R order
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r04i2; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_jt_tile.py -x -q --timeout 120 --timeout-method thread > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
tail -1 $o/t.log
timeout -k 10 300 python -u tools/tile_probe.py 125000 6016:16 > $o/probe.log 2>&1 || { tail -20 $o/probe.log; exit 1; }
grep "TLDS.*v5" $o/probe.log
FBN_JT_NO_LRU_ORDER=1 timeout -k 10 300 python -u tools/tile_probe.py 125000 6016:16 > $o/probe0.log 2>&1 || { tail -20 $o/probe0.log; exit 1; }
grep "TLDS.*v5" $o/probe0.log
