set -o pipefail
mkdir -p gpurun_out/r3g
timeout -k 10 400 python -u -m pytest tests/test_gpu_sgemm.py tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3g/tests.log 2>&1 || { tail -30 gpurun_out/r3g/tests.log; exit 1; }
tail -3 gpurun_out/r3g/tests.log
timeout -k 10 300 python -u tools/sgemm_bench.py > gpurun_out/r3g/sgemm.jsonl 2>&1 || exit 1
tail -4 gpurun_out/r3g/sgemm.jsonl
timeout -k 10 300 python -u tools/bench_extra.py c2train,mlmtrain > gpurun_out/r3g/train.jsonl 2>&1 || exit 1
cat gpurun_out/r3g/train.jsonl | tail -4
