#!/bin/bash
# Round profile evidence: bench line, rocprofv3 kernel stats of the same command, calibrated HBM
# traffic (FETCH_SIZE / WRITE_SIZE in separate --pmc passes) of the JT kernels and the CI kernels.
# usage: tools/profile_round.sh <outdir>
set -e
out=$1
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > $out/bench.json 2> $out/bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/stats -o run --output-format csv -- python -u bench.py --steps 10 --no-baseline > $out/stats_bench.json 2> $out/stats.err
cp $out/stats/run_kernel_stats.csv $out/kernel_stats.csv 2>/dev/null || find $out/stats -name "*kernel_stats.csv" -exec cp {} $out/kernel_stats.csv \;
bash tools/pmc_traffic.sh $out/traffic
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c -d $out/munin_$c -o pmc --output-format csv -- python tools/munin_once.py 125000 4 0 > $out/munin_$c.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc $c -d $out/pc5_$c -o pmc --output-format csv -- python tools/pc_probe.py 1000 100000 6 > $out/pc5_$c.log 2>&1
done
python tools/pmc_kernels.py $out > $out/pmc_kernels.json
