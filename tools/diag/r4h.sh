#!/bin/bash
# round 4 GPU session h: rocprofv3 kernel trace of the bench line, PMC passes (FETCH_SIZE,
# WRITE_SIZE, MFMA busy), trainer steps native vs RS_TRAIN_ROCBLAS=1 (interleaved)
set -eo pipefail
export TMPDIR=/tmp
O=gpurun_out/prof
rm -rf $O && mkdir -p $O
echo "[prof] kernel trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- \
    python bench.py --cpu-seconds 0 > $O/bench_under_rocprof.json 2> $O/kt.err
cp "$(find $O/kt -name '*kernel_stats.csv' | head -1)" $O/kernel_stats.csv
echo "[prof] pmc fetch"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- \
    python bench.py --utts 20 --steps 1 --warmup 0 --cpu-seconds 0 --no-profile --finetune-steps 0 > /dev/null 2> $O/fetch.err
echo "[prof] pmc write"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- \
    python bench.py --utts 20 --steps 1 --warmup 0 --cpu-seconds 0 --no-profile --finetune-steps 0 > /dev/null 2> $O/write.err
echo "[prof] pmc mfma"
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/mfma -o run --output-format csv -- \
    python bench.py --utts 20 --steps 1 --warmup 0 --cpu-seconds 0 --no-profile --finetune-steps 0 > /dev/null 2> $O/mfma.err
python tools/pmc_mfma.py "$(dirname "$(find $O/mfma -name '*counter_collection.csv' | head -1)")" $O/pmc_mfma.json > /dev/null
python tools/pmc_summary.py "$(dirname "$(find $O/fetch -name '*counter_collection.csv' | head -1)")" \
    "$(dirname "$(find $O/write -name '*counter_collection.csv' | head -1)")" $O/pmc_gemm_traffic.json > /dev/null
echo "[prof] trainer native vs rocblas"
for r in 1 2; do
  echo "## native_$r" >> $O/train_ab.txt
  timeout -k 10 300 python tools/bench_extra.py c2train,mlmtrain >> $O/train_ab.txt 2>> $O/train.err
  echo "## rocblas_$r" >> $O/train_ab.txt
  RS_TRAIN_ROCBLAS=1 timeout -k 10 300 python tools/bench_extra.py c2train,mlmtrain >> $O/train_ab.txt 2>> $O/train.err
done
cat $O/train_ab.txt
echo "[prof] done"
tail -c 1500 $O/bench_under_rocprof.json
