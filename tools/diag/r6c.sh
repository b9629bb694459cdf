#!/bin/bash
# Round 6: where the interleaved split-operand GEMM's time goes now — phase stamps (RS_DIAG build),
# the isolated-kernel variants (bare loop / no epilogue), and MFMA busy per kernel kind (PMC).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6c; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u tools/stamps.py 50 > $O/stamps.txt 2>&1 && \
PROBE=bare timeout -k 10 300 python -u tools/x3s_epi_probe.py 262144 3 > $O/probe_bare.txt 2>&1 && \
timeout -k 10 300 python -u tools/x3s_epi_probe.py 262144 3 > $O/probe_epi.txt 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/mfma -o run --output-format csv -- \
    python bench.py --utts 20 --steps 1 --warmup 0 --cpu-seconds 0 --no-profile --fp16-steps 0 --c4-secondary 0 --finetune-steps 0 > /dev/null 2> $O/mfma.err && \
python tools/pmc_mfma.py "$(dirname "$(find $O/mfma -name '*counter_collection.csv' | head -1)")" $O/pmc_mfma.json > $O/pmc_mfma.txt
rc=$?
cat $O/stamps.txt $O/probe_bare.txt $O/probe_epi.txt; cat $O/pmc_mfma.txt | head -30
exit $rc
