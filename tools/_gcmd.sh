set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_pc.py tests/test_gpu_pc_dist.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_pc.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/t_pc.log; exit 1; }
tail -1 gpurun_out/t_pc.log
echo "default"; timeout -k 10 120 python tools/pc5_timing.py 5 2>&1 | grep -E "run " | tail -1
timeout -k 10 120 python tools/pc_alarm_timing.py 2>&1 | tail -1
FBN_CI_BITSN=1 timeout -k 10 120 python tools/pc_alarm_timing.py 2>&1 | tail -1
mkdir -p gpurun_out/gl
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/gl -o run --output-format csv -- python tools/pc5_timing.py 3 > /dev/null 2>&1 || exit 1
python3 -c "
import csv
for r in list(csv.DictReader(open('gpurun_out/gl/run_kernel_stats.csv'))):
    if 'g2' in r['Name']: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us', round(float(r['TotalDurationNs'])/1e6/3,3), 'ms/run')
"
mkdir -p gpurun_out/gla
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/gla -o run --output-format csv -- python tools/pc_alarm_timing.py > /dev/null 2>&1 || exit 1
python3 -c "
import csv
for r in list(csv.DictReader(open('gpurun_out/gla/run_kernel_stats.csv')))[:8]:
    print('alarm', r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
