# trainer GEMM: new 128x64 configs (parity + timing) and a forced split-count sweep
set -o pipefail
mkdir -p gpurun_out/r3h




for s in 1 2 3 4 6; do
  SG_CFGS=0,5 RS_SGEMM_SPLITS=$s timeout -k 10 200 python -u tools/sgemm_bench.py > gpurun_out/r3h/split$s.jsonl 2>&1 || exit 1
  tail -1 gpurun_out/r3h/split$s.jsonl
done
