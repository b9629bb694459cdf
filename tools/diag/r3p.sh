# stream-K trainer GEMM: parity (all forms / shapes / configs, trainer suite), then timing vs torch
set -o pipefail
O=gpurun_out/r3p; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_sgemm.py tests/test_gpu_train.py -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
SG_CFGS=0,5 timeout -k 10 300 python -u tools/sgemm_bench.py > $O/sgemm.jsonl 2>&1 || { tail -20 $O/sgemm.jsonl; exit 1; }
tail -1 $O/sgemm.jsonl
RS_SGEMM_SK=0 SG_CFGS=0 timeout -k 10 300 python -u tools/sgemm_bench.py > $O/sgemm_nosk.jsonl 2>&1 || exit 1
tail -1 $O/sgemm_nosk.jsonl
timeout -k 10 300 python -u tools/bench_extra.py c2train,mlmtrain > $O/train.jsonl 2>&1 || exit 1
RS_TRAIN_ROCBLAS=1 timeout -k 10 300 python -u tools/bench_extra.py c2train,mlmtrain > $O/train_rocblas.jsonl 2>&1 || exit 1
grep workload $O/train.jsonl $O/train_rocblas.jsonl | cut -c1-220
