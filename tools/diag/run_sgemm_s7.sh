set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s7
for m in 1; do
  RS_SGEMM_MODE=$m timeout -k 10 300 python -u -m pytest tests/test_gpu_sgemm.py tests/test_gpu_train.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s7/test$m.log 2>&1 || { tail -30 gpurun_out/s7/test$m.log; exit 1; }
  echo "mode $m: $(tail -1 gpurun_out/s7/test$m.log)"
done
for m in 1; do
  RS_SGEMM_MODE=$m timeout -k 10 200 python -u tools/sgemm_bench.py > gpurun_out/s7/sgemm_m$m.jsonl 2>&1 || exit 1
  echo "mode $m: $(tail -1 gpurun_out/s7/sgemm_m$m.jsonl)"
  RS_SGEMM_MODE=$m timeout -k 10 200 python -u tools/bench_extra.py c2train,mlmtrain > gpurun_out/s7/train_m$m.jsonl 2>&1 || exit 1
  grep -v amdgpu gpurun_out/s7/train_m$m.jsonl | cut -c1-200
done
