#!/bin/bash
# round 6: split-count sweep of the software-pipelined trainer GEMM (cfg 12 / 14) against cfg 0 / 9 / 11
set -o pipefail
O=gpurun_out/r6x
rm -rf $O && mkdir -p $O
for sp in 1 2 3 4 6; do
  RS_SGEMM_SPLITS=$sp SG_CFGS=0,9,11,12,14 timeout -k 10 300 python -u tools/sgemm_bench.py > $O/split$sp.jsonl 2> $O/split$sp.err || exit $?
  tail -1 $O/split$sp.jsonl
done
SG_CFGS=0,9,11,12,14 timeout -k 10 300 python -u tools/sgemm_bench.py > $O/model.jsonl 2> $O/model.err
tail -1 $O/model.jsonl
