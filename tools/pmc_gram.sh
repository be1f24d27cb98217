set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc_g4
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d gpurun_out/pmc_g4/p1 -o pmc --output-format csv -- python3 tools/gram_timing.py 2 mfma > gpurun_out/pmc_g4/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_g4/p2 -o pmc --output-format csv -- python3 tools/gram_timing.py 2 mfma > gpurun_out/pmc_g4/p2.log 2>&1
for p in p1 p2; do grep -h "ci_gram_fp4" gpurun_out/pmc_g4/$p/pmc_counter_collection.csv | head -20 > gpurun_out/pmc_g4/$p.gram.csv; done
head -1 gpurun_out/pmc_g4/p1/pmc_counter_collection.csv
