#!/bin/bash
# Round-5 final PMC set (one counter group per rocprofv3 pass, each pass its own process under its
# own time limit; a crash fails the script, no masking):
#   ALARM headline kernel (tools/profile_r05.sh), Munin-like tiled kernel on 125k cases (FETCH /
#   WRITE + fp64 SQ pass), pc_small_kernel on ALARM-5000 (FETCH / WRITE), config-5 CI kernels
#   (tools/pc5_profile.sh), the copy8 calibration; then tools/r05_roofline_json.py assembles the
#   summaries bench.py reads (profiles/r05/*.json).
# usage: tools/profile_r05_final.sh <outdir>
set -e -o pipefail
out=$1
export TMPDIR=/tmp
mkdir -p $out/tp
bash tools/profile_r05.sh $out/alarm
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 240 rocprofv3 --pmc $c -d $out/tp/tile_$c -o pmc --output-format csv -- python tools/munin_once.py 125000 5 > $out/tp/tile_$c.log 2>&1
  timeout -k 10 120 rocprofv3 --pmc $c -d $out/tp/pcs_$c -o pmc --output-format csv -- python tools/pc_once.py 3 > $out/tp/pcs_$c.log 2>&1
  timeout -k 10 120 rocprofv3 --pmc $c -d $out/tp/cal_$c -o pmc --output-format csv -- ./tools/micro/calib_rw > $out/tp/cal_$c.log 2>&1
done
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_WAVES SQ_INSTS_LDS -d $out/tile_sq -o pmc --output-format csv -- python tools/munin_once.py 125000 5 > $out/tile_sq.log 2>&1
python tools/pmc_bytes.py $out/tp tile jt_tile_kernel 125000 > $out/tile_traffic.json
python tools/pmc_bytes.py $out/tp pcs pc_small_kernel > $out/pc_small_traffic.json
python tools/pmc_sq.py $out/tile_sq jt_tile_kernel > $out/tile_sq.json
bash tools/pc5_profile.sh $out/pc5
python tools/pmc_r02.py $out/pc5 > $out/pc5/pmc.json
python tools/pc5_kernels_json.py $out/pc5/pmc.json $out/pc5_kernels.json
echo profile done
