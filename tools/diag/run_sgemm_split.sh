set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s3
for t in 512 256 1024 128; do
  RS_SGEMM_SPLIT_WG=$t timeout -k 10 200 python -u tools/sgemm_bench.py > gpurun_out/s3/sgemm_split$t.jsonl 2>&1 || exit 1
  echo "target $t: $(tail -1 gpurun_out/s3/sgemm_split$t.jsonl)"
done
for t in 256 1024; do
  RS_SGEMM_SPLIT_WG=$t timeout -k 10 200 python -u tools/bench_extra.py c2train,mlmtrain > gpurun_out/s3/train_split$t.jsonl 2>&1 || exit 1
  echo "target $t:"; grep -v amdgpu gpurun_out/s3/train_split$t.jsonl | cut -c1-220
done
