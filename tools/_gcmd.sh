set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r02n; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_pc.py -x -q --timeout 300 --timeout-method thread -k "fused or level0 or config5" > $o/t1.log 2>&1 || { tail -30 $o/t1.log; exit 1; }
tail -1 $o/t1.log
for v in "FBN_CI_NO_FUSED0=1" "FBN_X=0"; do
  echo $v; env $v timeout -k 10 200 python tools/pc5_timing.py 8 2>&1 | grep "run " | tail -2 | sed 's/tests \[.*launched/launched/' || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/st -o run --output-format csv -- python tools/pc5_timing.py 3 > $o/st.log 2>&1 || { tail $o/st.log; exit 1; }
