#!/bin/bash
# Round-6 PMC set for the kernels this round changed (one counter group per rocprofv3 pass, each
# pass its own process under its own time limit; a crash fails the script):
#   ALARM headline kernel fbn_jt_gen with variable-major marginals (bench.py's layout) and, for
#   comparison, case-major: FETCH_SIZE / WRITE_SIZE (+ the copy8 calibration), one SQ pass (fp64
#   VALU) for the variable-major build; pc_small_kernel (ALARM-5000, level-1 information screen):
#   FETCH / WRITE; config-5 CI kernels (tools/pc5_profile.sh).  Then tools/r06_roofline_json.py
#   assembles the summaries bench.py reads (profiles/r06/*.json).
# usage: tools/profile_r06.sh <outdir>
set -e -o pipefail
out=$1
export TMPDIR=/tmp
mkdir -p $out/tp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $c -d $out/tp/alarm_$c -o pmc --output-format csv -- python tools/jt_once.py 3 0 3 100000 1 > $out/tp/alarm_$c.log 2>&1
  timeout -k 10 120 rocprofv3 --pmc $c -d $out/tp/alarmcm_$c -o pmc --output-format csv -- python tools/jt_once.py 3 0 3 100000 0 > $out/tp/alarmcm_$c.log 2>&1
  timeout -k 10 120 rocprofv3 --pmc $c -d $out/tp/pcs_$c -o pmc --output-format csv -- python tools/pc_once.py 3 > $out/tp/pcs_$c.log 2>&1
  timeout -k 10 120 rocprofv3 --pmc $c -d $out/tp/cal_$c -o pmc --output-format csv -- ./tools/micro/calib_rw > $out/tp/cal_$c.log 2>&1
done
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_WAVES SQ_INSTS_LDS -d $out/alarm_sq -o pmc --output-format csv -- python tools/jt_once.py 3 0 3 100000 1 > $out/alarm_sq.log 2>&1
python tools/pmc_bytes.py $out/tp alarm fbn_jt_gen 100000 > $out/alarm_traffic.json
python tools/pmc_bytes.py $out/tp alarmcm fbn_jt_gen 100000 > $out/alarm_cm_traffic.json
python tools/pmc_bytes.py $out/tp pcs pc_small_kernel > $out/pc_small_traffic.json
python tools/pmc_sq.py $out/alarm_sq fbn_jt_gen > $out/alarm_sq.json
bash tools/pc5_profile.sh $out/pc5
python tools/pmc_r02.py $out/pc5 > $out/pc5/pmc.json
python tools/pc5_kernels_json.py $out/pc5/pmc.json $out/pc5_kernels.json
echo profile done
