#!/bin/bash
# round 6: the trainer GEMM picker on the software-pipelined tile — parity (GEMM forms, trainer
# against autograd / the reference runs), the 27-shape sweep against torch, trainer steps native
# vs RS_TRAIN_ROCBLAS=1 (interleaved)
set -o pipefail
O=gpurun_out/r6z
rm -rf $O && mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sgemm.py tests/test_gpu_train.py > $O/tests.txt 2>&1
rc=$?
tail -3 $O/tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/sgemm_bench.py > $O/sgemm_all.jsonl 2> $O/sgemm_bench.err || exit $?
tail -1 $O/sgemm_all.jsonl
for r in 1 2; do
  echo "## native_$r" >> $O/train_ab.txt
  timeout -k 10 300 python tools/bench_extra.py c2train,mlmtrain >> $O/train_ab.txt 2>> $O/train.err || exit $?
  echo "## rocblas_$r" >> $O/train_ab.txt
  RS_TRAIN_ROCBLAS=1 timeout -k 10 300 python tools/bench_extra.py c2train,mlmtrain >> $O/train_ab.txt 2>> $O/train.err || exit $?
done
cat $O/train_ab.txt
