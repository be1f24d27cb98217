mkdir -p gpurun_out
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && timeout -k 10 300 python -u bench.py > gpurun_out/b1.json 2> gpurun_out/b1.err
