set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r03s2; mkdir -p $o
for cfg in "A FBN_PC_SYNC_SEPSETS=1 FBN_PC_PIPELINE_FULL=100000000" "B FBN_PC_PIPELINE_FULL=100000000" "C FBN_PC_SYNC_SEPSETS=1" "D X=1" "A2 FBN_PC_SYNC_SEPSETS=1 FBN_PC_PIPELINE_FULL=100000000"; do
  set -- $cfg; name=$1; shift
  env "$@" timeout -k 10 300 python -u tools/pc5_timing.py 20 > $o/ab_$name.log 2>&1 || { tail -20 $o/ab_$name.log; exit 1; }
  echo "$name $*: $(grep '^run' $o/ab_$name.log | tail -10 | awk '{print $4}' | sort -n | head -5 | tr '\n' ' ') | driver $(grep '^run' $o/ab_$name.log | tail -10 | awk '{print $7}' | sort -n | head -3 | tr '\n' ' ')"
done
