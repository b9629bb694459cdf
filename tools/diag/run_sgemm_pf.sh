set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s5
RS_SGEMM_PF=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_sgemm.py tests/test_gpu_train.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s5/test2.log 2>&1 || { tail -30 gpurun_out/s5/test2.log; exit 1; }
tail -2 gpurun_out/s5/test2.log
for st in 1 2; do
  RS_SGEMM_PF=$st timeout -k 10 200 python -u tools/sgemm_bench.py > gpurun_out/s5/sgemm_st$st.jsonl 2>&1 || exit 1
  echo "pf $st: $(tail -1 gpurun_out/s5/sgemm_st$st.jsonl)"
  RS_SGEMM_PF=$st timeout -k 10 200 python -u tools/bench_extra.py c2train,mlmtrain > gpurun_out/s5/train_st$st.jsonl 2>&1 || exit 1
  grep -v amdgpu gpurun_out/s5/train_st$st.jsonl | cut -c1-200
done
