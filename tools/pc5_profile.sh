#!/bin/bash
# Config-5 PC kernel profile (one MI355X): kernel trace + separate --pmc passes (FETCH_SIZE,
# WRITE_SIZE, SQ VALU counters) over tools/pc5_timing.py (3 PC-stable runs), calibrated with
# tools/micro/calib_rw.  usage: tools/pc5_profile.sh <outdir>; then
#   python tools/pmc_r02.py <outdir> > <outdir>/pmc.json && python tools/pc5_kernels_json.py <outdir>/pmc.json
set -o pipefail
out=$1
mkdir -p $out
export TMPDIR=/tmp
VALU="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
for c in FETCH_SIZE WRITE_SIZE VALU; do
  cc=$c; [ $c = VALU ] && cc="$VALU"
  timeout -k 10 120 rocprofv3 --pmc $cc -d $out/cal_$c -o pmc --output-format csv -- ./tools/micro/calib_rw > $out/cal_$c.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc $cc -d $out/pc5_$c -o pmc --output-format csv -- python tools/pc5_timing.py 3 > $out/pc5_$c.log 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/pc5_trace -o run --output-format csv -- python tools/pc5_timing.py 3 > $out/pc5_trace.log 2>&1 || exit 1
echo profile done
