# rocprofv3 kernel stats of the training benches (native k_sgemm GEMMs) -> gpurun_out/tprof
set -eo pipefail
export TMPDIR=/tmp
O=gpurun_out/tprof
rm -rf $O && mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- \
    python tools/bench_extra.py c2train,mlmtrain > $O/train_under_rocprof.jsonl 2> $O/kt.err
cp "$(find $O/kt -name '*kernel_stats.csv' | head -1)" $O/kernel_stats.csv
head -12 $O/kernel_stats.csv | cut -c1-200
