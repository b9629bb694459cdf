# persistent GEMM: swizzled epilogue slab (cfg 9 bias / 11 GELU) vs padded (13 / 14), then the
# stall/LDS-conflict counters of both
set -eo pipefail
export TMPDIR=/tmp
CFGS=9,13,11,14 DBGS=0 ROUNDS=3 timeout -k 10 300 python tools/gemm_bench.py 131072 > gpurun_out/epi_swz.txt 2>&1
CFGS=9,13 DBGS=0 SHAPES=2304x768 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_swz -o run -- python3 tools/gemm_bench.py 65536 > gpurun_out/pmc_swz.log 2>&1
