# scratch GPU command (gpurun): round-4 -- tiled kernel tests + PMC profiles
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r04n; mkdir -p $o
true

mkdir -p $o/prof
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $c -d $o/prof/pcs_$c -o pmc --output-format csv -- python tools/pc_once.py 3 > $o/prof/pcs_$c.log 2>&1 || grep -q "^ok" $o/prof/pcs_$c.log || exit 1
  timeout -k 10 120 rocprofv3 --pmc $c -d $o/prof/cal_$c -o pmc --output-format csv -- ./tools/micro/calib_rw > $o/prof/cal_$c.log 2>&1 || exit 1
done
python tools/pmc_bytes.py $o/prof pcs pc_small_kernel > $o/prof/pc_small_traffic.json
cat $o/prof/pc_small_traffic.json
