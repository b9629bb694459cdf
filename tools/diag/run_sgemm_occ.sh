set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s2
for o in 1 3 4; do
  RS_SGEMM_OCC=$o timeout -k 10 200 python -u tools/sgemm_bench.py > gpurun_out/s2/sgemm_occ$o.jsonl 2>&1 || exit 1
  tail -1 gpurun_out/s2/sgemm_occ$o.jsonl
done
