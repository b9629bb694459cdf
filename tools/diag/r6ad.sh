#!/bin/bash
# round 6: where the trainer steps spend their time (kernel stats of the c2train / mlmtrain legs)
set -eo pipefail
export TMPDIR=/tmp
O=gpurun_out/r6ad
rm -rf $O && mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c2 -o run --output-format csv -- \
    python tools/bench_extra.py c2train > $O/c2.jsonl 2> $O/c2.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/mlm -o run --output-format csv -- \
    python tools/bench_extra.py mlmtrain > $O/mlm.jsonl 2> $O/mlm.err
cp "$(find $O/c2 -name '*kernel_stats.csv' | head -1)" $O/c2_kernel_stats.csv
cp "$(find $O/mlm -name '*kernel_stats.csv' | head -1)" $O/mlm_kernel_stats.csv
cat $O/c2.jsonl $O/mlm.jsonl
