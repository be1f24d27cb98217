set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r02v; mkdir -p $o
timeout -k 10 400 python -u bench.py > $o/bench.json 2> $o/bench.err || { echo bench failed; tail -20 $o/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$o/bench.json').read().strip().splitlines()[-1]); print('value', d['value'], 'frac', d['roofline']['frac']); print({k:(d[k]['value'], d[k].get('ms_per_run', d[k].get('kernel_ms'))) for k in ('pc_stable','pc_synthetic','munin_like')})"
