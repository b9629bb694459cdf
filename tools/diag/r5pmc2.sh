#!/bin/bash
# Round 5: wave-state breakdown of the fp16x3 attention kernel (tools/attn_bench.py kind 10, C3-like lengths).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5pmc2; rm -rf $O; mkdir -p $O
KINDS=10 timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/db -o run -- python tools/attn_bench.py 7460 26 44 > $O/bench.txt 2> $O/prof.err || { tail -5 $O/prof.err; exit 1; }
python tools/diag/pmc_stall_summary.py $(find $O/db -name '*.db') > $O/stall.txt 2>&1; grep -i attn $O/stall.txt
rm -rf $O/db
