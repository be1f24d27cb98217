set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r02t; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
tail -1 $o/t.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { echo smoke failed; tail -20 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
timeout -k 10 400 python -u bench.py > $o/bench.json 2> $o/bench.err || { echo bench failed; tail -20 $o/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$o/bench.json').read().strip().splitlines()[-1]); print('value', d['value'], 'frac', d['roofline']['frac']); print({k:(d[k]['value'], d[k].get('ms_per_run', d[k].get('kernel_ms'))) for k in ('pc_stable','pc_synthetic','munin_like')})"
