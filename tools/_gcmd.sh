set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/profile_r02.sh gpurun_out/r02b || exit 1
python3 tools/pmc_r02.py gpurun_out/r02b > gpurun_out/r02b/pmc_r02b.json || exit 1
python3 tools/pc5_kernels_json.py gpurun_out/r02b/pmc_r02b.json gpurun_out/r02b/pc5_kernels.json
tail -c 300 gpurun_out/r02b/stats_bench.json
