set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pcprof
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pcprof/alarm -o run --output-format csv -- python tools/pc_alarm_timing.py > gpurun_out/pcprof/alarm.log 2>&1
cat gpurun_out/pcprof/alarm.log | tail -2
find gpurun_out/pcprof/alarm -name "*kernel_stats.csv" -exec cut -c1-200 {} \; | head -20
