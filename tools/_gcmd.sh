# scratch GPU command (gpurun): round-4 -- tiled kernel sweeps + fallback test
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r04k; mkdir -p $o
timeout -k 10 400 python -u tools/tile_probe.py 125000 6144:16 > $o/tile_probe.log 2>&1 || { tail -30 $o/tile_probe.log; exit 1; }
cat $o/tile_probe.log
