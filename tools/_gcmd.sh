set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_pc.py tests/test_gpu_pc_dist.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_pc.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/t_pc.log; exit 1; }
tail -1 gpurun_out/t_pc.log
for k in 1 2 4 8; do
mkdir -p gpurun_out/sk$k
FBN_CI_GRAM_SPLITK=$k timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/sk$k -o run --output-format csv -- python tools/pc5_timing.py 3 > gpurun_out/sk$k/out.log 2>&1 || exit 1
grep "run 2" gpurun_out/sk$k/out.log | cut -c1-60
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/sk$k/run_kernel_stats.csv')):
    if 'Cijk' in r['Name'] or 'sum_planes' in r['Name']: print('$k', r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
done
