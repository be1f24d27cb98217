set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r03s2; mkdir -p $o
timeout -k 10 600 python bench.py > $o/bench.json 2> $o/bench.err || { tail -20 $o/bench.err; exit 1; }
python -c "import json;d=json.load(open('$o/bench.json'));print(d['value'],d['ms_per_step'],d['pc_stable']['ms_per_run'],d['pc_stable']['kernel_ms_per_run'],d['pc_stable']['launched_per_level'],d['pc_synthetic']['ms_per_run'],d['pc_synthetic']['kernel_ms_per_run'],d['munin_like']['kernel_ms'])"
