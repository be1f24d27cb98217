set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r03s2; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_jt.py tests/test_gpu_jt_case.py -x -q --timeout 200 --timeout-method thread > $o/jt_t.log 2>&1 || { tail -40 $o/jt_t.log; exit 1; }
tail -2 $o/jt_t.log
timeout -k 10 400 python -u tools/case_probe.py 125000 4 > $o/probe.log 2>&1 || { tail -20 $o/probe.log; exit 1; }
cat $o/probe.log | grep variant
timeout -k 10 600 python -u tools/jt_budget_sweep.py "200:96,190:96,180:96,160:96,200:88,200:104" > $o/budget.log 2>&1 || { tail -20 $o/budget.log; exit 1; }
grep budget $o/budget.log
