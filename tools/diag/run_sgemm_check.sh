set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s1
timeout -k 10 400 python -u -m pytest tests/test_gpu_sgemm.py tests/test_gpu_train.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s1/test.log 2>&1 || { tail -40 gpurun_out/s1/test.log; exit 1; }
tail -5 gpurun_out/s1/test.log
timeout -k 10 200 python -u tools/sgemm_bench.py > gpurun_out/s1/sgemm.jsonl 2>&1 || exit 1
cat gpurun_out/s1/sgemm.jsonl
timeout -k 10 200 python -u tools/bench_extra.py c2train,mlmtrain > gpurun_out/s1/train_native.jsonl 2>&1 || exit 1
RS_TRAIN_ROCBLAS=1 timeout -k 10 200 python -u tools/bench_extra.py c2train,mlmtrain > gpurun_out/s1/train_rocblas.jsonl 2>&1 || exit 1
cat gpurun_out/s1/train_native.jsonl gpurun_out/s1/train_rocblas.jsonl
