#!/bin/bash
# Round 6: the PMC passes of profile_round.sh alone (MFMA busy first, then FETCH_SIZE, WRITE_SIZE).
set -eo pipefail
export TMPDIR=/tmp
O=gpurun_out/prof2; rm -rf $O; mkdir -p $O
A="--utts 20 --steps 1 --warmup 0 --cpu-seconds 0 --no-profile --c4-secondary 0 --fp16-steps 0 --finetune-steps 0"
echo "[pmc] mfma"
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/mfma -o run --output-format csv -- python bench.py $A > /dev/null 2> $O/mfma.err
python tools/pmc_mfma.py "$(dirname "$(find $O/mfma -name '*counter_collection.csv' | head -1)")" $O/pmc_mfma.json > /dev/null
echo "[pmc] fetch"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python bench.py $A > /dev/null 2> $O/fetch.err
echo "[pmc] write"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python bench.py $A > /dev/null 2> $O/write.err
python tools/pmc_summary.py "$(dirname "$(find $O/fetch -name '*counter_collection.csv' | head -1)")" \
    "$(dirname "$(find $O/write -name '*counter_collection.csv' | head -1)")" $O/pmc_gemm_traffic.json > /dev/null
echo "[pmc] done"
