#!/bin/bash
# Round 5: wave-state breakdown of the split-operand GEMM variants (prod / nowait / alias / noepi) at
# the FFN1 and BertOutput shapes: one PMC pass (8 SQ + 1 GRBM counters), tools/diag/pmc_stall_summary.py.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5pmc; rm -rf $O; mkdir -p $O
SHAPES=3072x768,768x3072 timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/db -o run -- python tools/x3s_epi_probe.py 262144 2 > $O/probe.txt 2> $O/prof.err || { tail -5 $O/prof.err; exit 1; }
python tools/diag/pmc_stall_summary.py $(find $O/db -name '*.db') > $O/stall.txt 2>&1; cat $O/stall.txt
rm -rf $O/db
