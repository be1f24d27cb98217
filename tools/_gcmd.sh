# scratch GPU command (gpurun): round-4 -- tiled kernel at 5 waves per SIMD (U = 2 for >= 4 factors)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r04n2; mkdir -p $o
timeout -k 10 300 python -u tools/tile_probe.py 125000 3968:20 6016:16 > $o/probe.log 2>&1 || { tail -20 $o/probe.log; exit 1; }
grep "TLDS.*v5" $o/probe.log
