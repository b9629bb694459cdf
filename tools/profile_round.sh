#!/bin/bash
# One GPU call: full bench line + rocprofv3 kernel stats of the same workload + separate
# FETCH_SIZE / WRITE_SIZE PMC passes (MI355X_MICROARCH.md HBM recipe) -> gpurun_out/prof/.
# usage (on the GPU box, repo root): bash tools/profile_round.sh
# (the PMC passes skip the fine-tune / C4 / fp16 legs: with the trainer's ~100k dispatches before the
# scoring launches, rocprofv3 --pmc itself segfaulted in the x3s launch once in round 6; without them
# every pass completes — gpurun_out/prof vs prof2)
set -eo pipefail
export TMPDIR=/tmp
O=gpurun_out/prof
rm -rf $O && mkdir -p $O
echo "[prof] bench"
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err
echo "[prof] kernel trace"
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- \
    python bench.py --cpu-seconds 0 --c4-secondary 0 --fp16-steps 0 > $O/bench_under_rocprof.json 2> $O/kt.err
echo "[prof] pmc fetch"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- \
    python bench.py --utts 20 --steps 1 --warmup 0 --cpu-seconds 0 --no-profile --c4-secondary 0 --fp16-steps 0 --finetune-steps 0 > /dev/null 2> $O/fetch.err
echo "[prof] pmc write"
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- \
    python bench.py --utts 20 --steps 1 --warmup 0 --cpu-seconds 0 --no-profile --c4-secondary 0 --fp16-steps 0 --finetune-steps 0 > /dev/null 2> $O/write.err
echo "[prof] pmc mfma"
timeout -k 10 600 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/mfma -o run --output-format csv -- \
    python bench.py --utts 20 --steps 1 --warmup 0 --cpu-seconds 0 --no-profile --c4-secondary 0 --fp16-steps 0 --finetune-steps 0 > /dev/null 2> $O/mfma.err
python tools/pmc_mfma.py "$(dirname "$(find $O/mfma -name '*counter_collection.csv' | head -1)")" $O/pmc_mfma.json > /dev/null
echo "[prof] extra configs"
timeout -k 10 900 python tools/bench_extra.py > $O/bench_extra.jsonl 2> $O/extra.err
python tools/pmc_summary.py "$(dirname "$(find $O/fetch -name '*counter_collection.csv' | head -1)")" \
    "$(dirname "$(find $O/write -name '*counter_collection.csv' | head -1)")" $O/pmc_gemm_traffic.json > /dev/null
cp "$(find $O/kt -name '*kernel_stats.csv' | head -1)" $O/kernel_stats.csv
echo "[prof] done"
tail -c 2000 $O/bench.json
