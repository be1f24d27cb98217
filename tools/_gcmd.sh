set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/r02k; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_pc.py -x -q --timeout 300 --timeout-method thread > $o/t1.log 2>&1 || { tail -30 $o/t1.log; exit 1; }
tail -1 $o/t1.log
timeout -k 10 200 python tools/pc5_timing.py 6 2>&1 | grep "run " | tail -2 || exit 1
timeout -k 10 120 python tools/pc_alarm_cabi.py 200 "alarm" 2>&1 | tail -1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/st -o run --output-format csv -- python tools/pc5_timing.py 3 > $o/st.log 2>&1 || { tail $o/st.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/sta -o run --output-format csv -- python tools/pc_alarm_cabi.py 50 x > $o/sta.log 2>&1 || { tail $o/sta.log; exit 1; }
