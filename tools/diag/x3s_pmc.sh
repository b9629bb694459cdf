# x3s GEMM: timing variants + SQ stall breakdown (GPU box, repo root): bash tools/diag/x3s_pmc.sh <tag>
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python -u tools/x3s_bench.py 131072 > $O/bench.txt 2>&1 || exit $?
grep -v amdgpu.ids $O/bench.txt
export SHAPES=2304x768,768x3072 VARIANTS=x3s-f32,x3s-f32-ilv,x3s-f32-neither,kcat-persist-f16
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc -o run -- python3 tools/x3s_bench.py 65536 > $O/pmc.log 2>&1 || exit $?
python3 tools/diag/pmc_stall_summary.py $(find $O/pmc -name '*.db' | head -1) | tee $O/stall.txt
