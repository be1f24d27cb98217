#!/bin/bash
# VALU work of the JT kernels per launch (rocprofv3 SQ counters, one --pmc pass per program):
# ALARM specialized kernel (100k cases) and the Munin-like streamed kernel (125k cases).
# usage: tools/pmc_valu.sh <outdir>
set -e
out=$1
export TMPDIR=/tmp
mkdir -p $out
C="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
timeout -s KILL 120 rocprofv3 --pmc $C -d $out/alarm -o pmc --output-format csv -- python tools/jt_once.py -1 0 3 > $out/alarm.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc $C -d $out/munin -o pmc --output-format csv -- python tools/munin_once.py 125000 4 0 > $out/munin.log 2>&1
python tools/pmc_summary.py $out/alarm fbn_jt_gen > $out/alarm_valu.txt
python tools/pmc_summary.py $out/munin jt_virt > $out/munin_valu.txt
cat $out/alarm_valu.txt $out/munin_valu.txt
