set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r03s2; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_jt_case.py -x -q --timeout 120 --timeout-method thread > $o/case.log 2>&1 || { tail -40 $o/case.log; exit 1; }
tail -2 $o/case.log
timeout -k 10 400 python -u tools/case_probe.py 125000 4,5 8,12,16 0,7 > $o/probe.log 2>&1 || { tail -20 $o/probe.log; exit 1; }
cat $o/probe.log
timeout -k 10 300 python -u tools/case_prof.py 125000 12 > $o/prof.log 2>&1 || { tail -20 $o/prof.log; exit 1; }
cat $o/prof.log
