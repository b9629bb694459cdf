#!/bin/bash
# round 6: wide / fused LayerNorm column sums in the trainer — trainer parity, step timing, kernel stats
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6ae
rm -rf $O && mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_cli.py > $O/tests.txt 2>&1
rc=$?
tail -3 $O/tests.txt
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  echo "## native_$r" >> $O/train_ab.txt
  timeout -k 10 300 python tools/bench_extra.py c2train,mlmtrain >> $O/train_ab.txt 2>> $O/train.err || exit $?
  echo "## rocblas_$r" >> $O/train_ab.txt
  RS_TRAIN_ROCBLAS=1 timeout -k 10 300 python tools/bench_extra.py c2train,mlmtrain >> $O/train_ab.txt 2>> $O/train.err || exit $?
done
cat $O/train_ab.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/mlm -o run --output-format csv -- \
    python tools/bench_extra.py mlmtrain > $O/mlm.jsonl 2> $O/mlm.err
cp "$(find $O/mlm -name '*kernel_stats.csv' | head -1)" $O/mlm_kernel_stats.csv
