#!/bin/bash
# HBM traffic of the JT kernel per launch (rocprofv3 FETCH_SIZE / WRITE_SIZE, one counter per pass,
# no tracing domains mixed in), calibrated with a known-byte 8-B/lane copy kernel.
# usage: tools/pmc_traffic.sh <outdir>     (writes <outdir>/traffic.json)
set -e
out=$1
export TMPDIR=/tmp
mkdir -p $out
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 240 rocprofv3 --pmc $c -d $out/jt_$c -o pmc --output-format csv -- python tools/jt_once.py -1 0 3 > $out/jt_$c.log 2>&1
  timeout -k 10 120 rocprofv3 --pmc $c -d $out/cal_$c -o pmc --output-format csv -- ./tools/micro/calib_rw > $out/cal_$c.log 2>&1
done
python tools/traffic_json.py $out > $out/traffic.json
cat $out/traffic.json
