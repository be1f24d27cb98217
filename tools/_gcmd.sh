set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r03s2; mkdir -p $o
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
tail -1 $o/t.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { echo smoke failed; tail -20 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
timeout -k 10 700 python bench.py > $o/bench.json 2> $o/bench.err || { tail -20 $o/bench.err; exit 1; }
python -c "import json;d=json.load(open('$o/bench.json'));print(d['value'],d['ms_per_step'],d['pc_stable']['ms_per_run'],d['pc_stable']['kernel_ms_per_run'],d['pc_synthetic']['ms_per_run'],d['pc_synthetic']['kernel_ms_per_run'],d['munin_like']['kernel_ms'])"
