set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r02c_prof; mkdir -p $o
timeout -k 10 400 python -u bench.py > $o/bench.json 2> $o/bench.err || { echo bench failed; tail -20 $o/bench.err; exit 1; }
echo bench ok
bash tools/profile_r02.sh $o || { echo profile failed; exit 1; }
