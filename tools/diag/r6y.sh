#!/bin/bash
# round 6: trainer GEMM with 2 / 3 / 4 LDS stages (cfg 12-16): parity, then a split-count sweep
set -o pipefail
O=gpurun_out/r6y
rm -rf $O && mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sgemm.py > $O/sgemm_tests.txt 2>&1
rc=$?
tail -3 $O/sgemm_tests.txt
[ $rc -eq 0 ] || exit $rc
for sp in 1 2 3 4 6; do
  RS_SGEMM_SPLITS=$sp SG_CFGS=0,11,12,13,14,15,16 timeout -k 10 300 python -u tools/sgemm_bench.py > $O/split$sp.jsonl 2> $O/split$sp.err || exit $?
  tail -1 $O/split$sp.jsonl
done
