set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
cp fastbn_amd/libfastbn.so /tmp/libfastbn_w3.so
for w in w3 w4 w5; do
  cp /tmp/libfastbn_$w.so fastbn_amd/libfastbn.so 2>/dev/null || cp fastbn_amd/libfastbn_$w.so fastbn_amd/libfastbn.so
  echo $w; timeout -k 10 200 python tools/pc5_timing.py 6 2>&1 | grep "run " | tail -2 | sed 's/tests \[.*launched/launched/' || exit 1
  mkdir -p gpurun_out/r02l_$w
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02l_$w -o run --output-format csv -- python tools/pc5_timing.py 3 > /dev/null 2>&1 || exit 1
done
cp /tmp/libfastbn_w3.so fastbn_amd/libfastbn.so
