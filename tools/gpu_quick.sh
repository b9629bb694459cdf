#!/bin/bash
# Quick GPU check: fp16x3 C3 bench line + rocprofv3 kernel stats of a short run.
# usage (GPU box, repo root): bash tools/gpu_quick.sh <tag> [bench args...]
set -eo pipefail
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG
rm -rf $O && mkdir -p $O
echo "[quick] bench"
timeout -k 10 600 python -u bench.py "$@" > $O/bench.json 2> $O/bench.err
tail -c 3000 $O/bench.json
echo "[quick] kernel trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- \
    python bench.py --steps 1 --warmup 1 --cpu-seconds 0 --fp16-steps 0 --utts 50 "$@" > $O/bench_under_rocprof.json 2> $O/kt.err
cp "$(find $O/kt -name '*kernel_stats.csv' | head -1)" $O/kernel_stats.csv
head -20 $O/kernel_stats.csv | cut -c1-250
echo "[quick] done"
