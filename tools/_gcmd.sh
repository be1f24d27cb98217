timeout -k 10 300 python -u bench.py --steps 10 > gpurun_out/b1.json 2> gpurun_out/b1.err
