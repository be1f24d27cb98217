# scratch GPU command (gpurun): round-4 -- ALARM fast-order kernel: codegen settings sweep + PMC
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r04s; mkdir -p $o/prof
timeout -k 10 400 python -u tools/jt_env_sweep.py ":4" ":8" "FBN_JT_MIN_WAVES=2:8" "FBN_JT_MIN_WAVES=2,FBN_JT_PREFETCH_BUDGET=100:8" \
  "FBN_JT_REG_ENTRIES=128:4" "FBN_JT_PREFETCH_BUDGET=300:4" "FBN_JT_MIN_WAVES=2,FBN_JT_REG_ENTRIES=64:8" "FBN_JT_PREFETCH_BUDGET=120:4" > $o/sweep.log 2>&1 || { tail -20 $o/sweep.log; exit 1; }
cat $o/sweep.log
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $c -d $o/prof/alarm_$c -o pmc --output-format csv -- python tools/jt_once.py -1 0 3 > $o/prof/alarm_$c.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc $c -d $o/prof/cal_$c -o pmc --output-format csv -- ./tools/micro/calib_rw > $o/prof/cal_$c.log 2>&1 || exit 1
done
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d $o/prof/alarm_sq -o pmc --output-format csv -- python tools/jt_once.py -1 0 3 > $o/prof/alarm_sq.log 2>&1 || exit 1
python tools/pmc_bytes.py $o/prof alarm fbn_jt_gen 100000 > $o/prof/alarm_traffic.json
python tools/pmc_summary.py $o/prof/alarm_sq fbn_jt_gen | tee $o/prof/alarm_valu.txt
cat $o/prof/alarm_traffic.json
