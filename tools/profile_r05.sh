#!/bin/bash
# Round-5 PMC of the ALARM headline kernel (fbn_jt_gen, variant 3, 100k cases, tools/jt_once.py):
# FETCH_SIZE and WRITE_SIZE in passes of their own + the copy8 calibration (tools/micro/calib_rw),
# and one SQ pass with the fp64 instruction counters (the VALU roofline of bench.py).  Every pass
# is its own process under its own time limit; a crash fails the script (no masking).
# usage: tools/profile_r05.sh <outdir>
set -e -o pipefail
out=$1
export TMPDIR=/tmp
mkdir -p $out
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $c -d $out/alarm_$c -o pmc --output-format csv -- python tools/jt_once.py 3 0 3 > $out/alarm_$c.log 2>&1
  timeout -k 10 120 rocprofv3 --pmc $c -d $out/cal_$c -o pmc --output-format csv -- ./tools/micro/calib_rw > $out/cal_$c.log 2>&1
done
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_WAVES SQ_INSTS_LDS -d $out/alarm_sq -o pmc --output-format csv -- python tools/jt_once.py 3 0 3 > $out/alarm_sq.log 2>&1
python tools/pmc_bytes.py $out alarm fbn_jt_gen 100000 > $out/alarm_traffic.json
python tools/pmc_sq.py $out/alarm_sq fbn_jt_gen > $out/alarm_sq.json
cat $out/alarm_traffic.json $out/alarm_sq.json
