# scratch GPU command (gpurun): full GPU suite + default bench line of the committed tree
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r03s3; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gpu_all2.log 2>&1 || { tail -40 $o/gpu_all2.log; exit 1; }
tail -1 $o/gpu_all2.log
timeout -k 10 900 python -u bench.py > $o/bench2.json 2> $o/bench2.err || { tail -30 $o/bench2.err; exit 1; }
echo bench done
