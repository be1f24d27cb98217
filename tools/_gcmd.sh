# scratch GPU command (gpurun): full GPU suite + smoke on the committed tree
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r03s3; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gpu_all.log 2>&1 || { tail -40 $o/gpu_all.log; exit 1; }
tail -1 $o/gpu_all.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.log 2>&1 || { tail -30 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
