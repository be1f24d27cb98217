#!/bin/bash
# Round-4 PMC profiles (one counter group per rocprofv3 pass, nothing else mixed in):
#   tiled JT kernel on 125k Munin-like cases (FETCH/WRITE + SQ instruction / cycle counters),
#   pc_small_kernel on ALARM-5000 (FETCH/WRITE), the copy8 calibration.
# usage: tools/profile_r04.sh <outdir>
set -e
out=$1
export TMPDIR=/tmp
mkdir -p $out
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 240 rocprofv3 --pmc $c -d $out/tile_$c -o pmc --output-format csv -- python tools/munin_once.py 125000 5 > $out/tile_$c.log 2>&1
  # (round 5: no exit mask -- a crash in the process's teardown fails the script)
  timeout -k 10 120 rocprofv3 --pmc $c -d $out/pcs_$c -o pmc --output-format csv -- python tools/pc_once.py 3 > $out/pcs_$c.log 2>&1
  timeout -k 10 120 rocprofv3 --pmc $c -d $out/cal_$c -o pmc --output-format csv -- ./tools/micro/calib_rw > $out/cal_$c.log 2>&1
done
for c in FETCH_SIZE WRITE_SIZE; do :; done
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_INST_CYCLES_SMEM"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp -d $out/sq$i -o pmc --output-format csv -- python tools/munin_once.py 125000 5 > $out/sq$i.log 2>&1
done
python tools/pmc_bytes.py $out tile jt_tile_kernel 125000 > $out/tile_traffic.json
python tools/pmc_bytes.py $out pcs pc_small_kernel > $out/pc_small_traffic.json
cat $out/tile_traffic.json $out/pc_small_traffic.json
