#!/bin/bash
# round 6: picker with the half tiles (cfg 17 / 18) — the 27-shape sweep against torch (x2)
set -o pipefail
O=gpurun_out/r6ab
rm -rf $O && mkdir -p $O
for r in 1 2; do
  SG_CFGS=11,12,17 timeout -k 10 300 python -u tools/sgemm_bench.py > $O/sgemm_all_$r.jsonl 2> $O/sgemm_bench_$r.err || exit $?
  tail -1 $O/sgemm_all_$r.jsonl
done
