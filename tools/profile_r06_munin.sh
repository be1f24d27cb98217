#!/bin/bash
# Round-6 PMC of the Munin-like tiled kernel after the branch-free factor loads (jt_tile.hip
# FBN_TILE_REUSE=0): FETCH_SIZE / WRITE_SIZE (+ the copy8 calibration) and one SQ pass, one counter
# group per rocprofv3 pass, each its own process under its own time limit; then
# tools/r06_munin_json.py writes profiles/r06/munin_traffic.json and the "munin" entry of
# profiles/r06/jt_valu.json (the summaries bench.py reads).  usage: tools/profile_r06_munin.sh <outdir>
set -e -o pipefail
out=$1
export TMPDIR=/tmp
mkdir -p $out/tp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 240 rocprofv3 --pmc $c -d $out/tp/tile_$c -o pmc --output-format csv -- python tools/munin_once.py 125000 5 > $out/tp/tile_$c.log 2>&1
  timeout -k 10 120 rocprofv3 --pmc $c -d $out/tp/cal_$c -o pmc --output-format csv -- ./tools/micro/calib_rw > $out/tp/cal_$c.log 2>&1
done
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_WAVES SQ_INSTS_LDS -d $out/tile_sq -o pmc --output-format csv -- python tools/munin_once.py 125000 5 > $out/tile_sq.log 2>&1
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $out/tile_sq2 -o pmc --output-format csv -- python tools/munin_once.py 125000 5 > $out/tile_sq2.log 2>&1
python tools/pmc_bytes.py $out/tp tile jt_tile_kernel 125000 > $out/tile_traffic.json
python tools/pmc_sq.py $out/tile_sq jt_tile_kernel > $out/tile_sq.json
python tools/pmc_sq.py $out/tile_sq2 jt_tile_kernel > $out/tile_sq2.json
echo profile done
