#!/bin/bash
# Round-3 second-session profile evidence (one MI355X): rocprofv3 kernel stats of the bench command
# and calibrated FETCH_SIZE / WRITE_SIZE passes over the ALARM-5000 PC call loop (device-resident
# search, pc_small.hip).  usage: tools/profile_s2.sh <outdir>
set -o pipefail
out=$1
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/stats -o run --output-format csv -- python -u bench.py --steps 10 --no-baseline --no-loaders > $out/stats_bench.json 2> $out/stats.err || exit 1
echo "stats done"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d $out/cal_$c -o pmc --output-format csv -- ./tools/micro/calib_rw > $out/cal_$c.log 2>&1 || exit 1
  timeout -s KILL 200 rocprofv3 --pmc $c -d $out/pcsmall_$c -o pmc --output-format csv -- python tools/pc_small_timing.py 20 > $out/pcsmall_$c.log 2>&1 || exit 1
  echo "pmc $c done"
done
