set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_pc_dist.py tests/test_gpu_pc.py -x -v --timeout 300 --timeout-method thread > gpurun_out/t_dist.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_dist.log; exit 1; }
tail -3 gpurun_out/t_dist.log
FBN_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --no-munin > gpurun_out/b2.json 2> gpurun_out/b2.err || { echo "bench2 failed"; tail -30 gpurun_out/b2.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/b2.json'));print(json.dumps(d['pc_synthetic'],indent=0)[:1500])"
