#!/bin/bash
# trainer GEMM: 192x128 config + time-model picker: parity (sgemm forms, trainer suite), sweep vs
# rocBLAS, then training steps native vs RS_TRAIN_ROCBLAS=1 interleaved (two rounds)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3u; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_sgemm.py tests/test_gpu_train.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1
rc=$?; tail -3 $O/test.log; [ $rc -ne 0 ] && exit $rc
SG_CFGS=0,9,10 timeout -k 10 400 python -u tools/sgemm_bench.py > $O/sweep.jsonl 2> $O/sweep.err || exit 1
tail -1 $O/sweep.jsonl
for r in 1; do
  timeout -k 10 300 python -u tools/bench_extra.py c2train,mlmtrain > $O/train_native_$r.jsonl 2>&1 || exit 1
  RS_TRAIN_ROCBLAS=1 timeout -k 10 300 python -u tools/bench_extra.py c2train,mlmtrain > $O/train_rocblas_$r.jsonl 2>&1 || exit 1
done
grep -h workload $O/train_*.jsonl | cut -c1-200
