# scratch GPU command (gpurun): round-4 -- full GPU suite, bench, kernel-trace stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r04z; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $o/gpu_tests.log 2>&1 || { tail -30 $o/gpu_tests.log; exit 1; }
tail -2 $o/gpu_tests.log
timeout -k 10 600 python bench.py > $o/bench.json 2> $o/bench.err || { tail -20 $o/bench.err; exit 1; }
python -c "import json;d=json.loads(open('$o/bench.json').read().strip().splitlines()[-1]);print(json.dumps(d['summary']))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/ktrace -o kt --output-format csv -- python bench.py --steps 5 --no-baseline --no-loaders > $o/kt_bench.json 2> $o/kt_bench.err || { tail -5 $o/kt_bench.err; exit 1; }
ls $o/ktrace
