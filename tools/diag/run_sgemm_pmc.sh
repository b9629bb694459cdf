# stall / LDS / MFMA-busy counters of the trainer GEMM over tools/sgemm_bench.py (one PMC pass)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/sgpmc; rm -rf gpurun_out/sgpmc/db
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/sgpmc/db -o run -- python3 tools/sgemm_bench.py > gpurun_out/sgpmc/run.log 2>&1 || exit 1
python3 tools/diag/pmc_stall_summary.py $(find gpurun_out/sgpmc/db -name '*.db' | head -1) > gpurun_out/sgpmc/summary.txt 2>&1 || { find gpurun_out/sgpmc/db | head; exit 1; }
cat gpurun_out/sgpmc/summary.txt
rm -rf gpurun_out/sgpmc/db
