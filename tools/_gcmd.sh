set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 60 ./tools/micro/valu_rate
bash tools/pc5_profile.sh gpurun_out/prof_pc5 || exit 1
python3 tools/pmc_r02.py gpurun_out/prof_pc5 > gpurun_out/prof_pc5/pmc.json && python3 tools/pc5_kernels_json.py gpurun_out/prof_pc5/pmc.json gpurun_out/prof_pc5/pc5_kernels.json
