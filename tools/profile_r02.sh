#!/bin/bash
# Round-2 profile evidence (one MI355X): rocprofv3 kernel stats of the bench command, and per-kernel
# PMC counters in separate passes (FETCH_SIZE, WRITE_SIZE, SQ VALU counters; no tracing domains
# mixed in) for the ALARM JT kernel, the Munin-like streamed kernel and the config-5 PC kernels,
# calibrated with a known-byte copy kernel (tools/micro/calib_rw).
# usage: tools/profile_r02.sh <outdir>      (then: python tools/pmc_r02.py <outdir>)
set -o pipefail
out=$1
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/stats -o run --output-format csv -- python -u bench.py --steps 10 --no-baseline --no-loaders > $out/stats_bench.json 2> $out/stats.err || exit 1
VALU="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
for c in FETCH_SIZE WRITE_SIZE VALU; do
  cc=$c; [ $c = VALU ] && cc="$VALU"
  timeout -k 10 120 rocprofv3 --pmc $cc -d $out/cal_$c -o pmc --output-format csv -- ./tools/micro/calib_rw > $out/cal_$c.log 2>&1 || exit 1
  timeout -k 10 200 rocprofv3 --pmc $cc -d $out/alarm_$c -o pmc --output-format csv -- python tools/jt_once.py -1 0 3 > $out/alarm_$c.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc $cc -d $out/munin_$c -o pmc --output-format csv -- python tools/munin_once.py 125000 -1 0 > $out/munin_$c.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc $cc -d $out/pc5_$c -o pmc --output-format csv -- python tools/pc5_timing.py 3 > $out/pc5_$c.log 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/pc5_trace -o run --output-format csv -- python tools/pc5_timing.py 3 > $out/pc5_trace.log 2>&1 || exit 1
echo profile done
