# scratch GPU command (gpurun): round-4 -- pc_small plain launch default
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r04h2; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_pc_small.py tests/test_gpu_pc_dist.py tests/test_gpu_cli.py -x -v --timeout 120 --timeout-method thread > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
tail -1 $o/t.log
timeout -k 10 300 python -u tools/pc_small_timing.py 400 > $o/tm.log 2>&1 || { tail -20 $o/tm.log; exit 1; }
grep median $o/tm.log
