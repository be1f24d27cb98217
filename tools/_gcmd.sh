set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r02d_prof; mkdir -p $o
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { echo smoke failed; tail -20 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
timeout -k 10 400 python -u bench.py > $o/bench.json 2> $o/bench.err || { echo bench failed; tail -20 $o/bench.err; exit 1; }
echo bench ok
bash tools/profile_r02.sh $o || { echo profile failed; exit 1; }
