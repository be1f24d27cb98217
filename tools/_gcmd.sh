# scratch GPU command (gpurun): round-4 -- N = 2 rehearsal (gloo, ranks share the GPU) incl. Munin-like
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r04u2; mkdir -p $o
FBN_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29543 bench.py --gpus 2 --steps 3 --warmup 1 --no-loaders --no-baseline > $o/b2.json 2> $o/b2.err || { tail -20 $o/b2.err; exit 1; }
python -c "import json;d=json.loads(open('$o/b2.json').read().strip().splitlines()[-1]);print(json.dumps(d['summary']))"
