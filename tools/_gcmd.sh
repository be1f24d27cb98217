mkdir -p gpurun_out
FBN_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 > gpurun_out/b2.json 2> gpurun_out/b2.err && timeout -k 10 300 python -u bench.py --steps 5 --no-pc --no-baseline > gpurun_out/b1.json 2> gpurun_out/b1.err
