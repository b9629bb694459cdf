#!/bin/bash
# round 6: final trainer GEMM picker (cfg 11 one-pass model, half tiles) — parity, sweep x2, trainer A/B
set -o pipefail
O=gpurun_out/r6ac
rm -rf $O && mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sgemm.py tests/test_gpu_train.py > $O/tests.txt 2>&1
rc=$?
tail -3 $O/tests.txt
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  SG_CFGS=11,12,17 timeout -k 10 300 python -u tools/sgemm_bench.py > $O/sgemm_all_$r.jsonl 2> $O/sgemm_bench_$r.err || exit $?
  tail -1 $O/sgemm_all_$r.jsonl
done
for r in 1 2; do
  echo "## native_$r" >> $O/train_ab.txt
  timeout -k 10 300 python tools/bench_extra.py c2train,mlmtrain >> $O/train_ab.txt 2>> $O/train.err || exit $?
  echo "## rocblas_$r" >> $O/train_ab.txt
  RS_TRAIN_ROCBLAS=1 timeout -k 10 300 python tools/bench_extra.py c2train,mlmtrain >> $O/train_ab.txt 2>> $O/train.err || exit $?
done
cat $O/train_ab.txt
