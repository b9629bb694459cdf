#!/bin/bash
# round 6: smaller software-pipelined trainer tiles (cfg 17-19: 64x128, 128x64, 64x64) for the
# ~1k-token GEMMs — parity, then a split sweep at 1100 tokens against cfg 11 / 12
set -o pipefail
O=gpurun_out/r6aa
rm -rf $O && mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sgemm.py > $O/tests.txt 2>&1
rc=$?
tail -3 $O/tests.txt
[ $rc -eq 0 ] || exit $rc
for sp in 1 2 3 4 6; do
  SG_TOKENS=1100 RS_SGEMM_SPLITS=$sp SG_CFGS=11,12,17,18,19 timeout -k 10 300 python -u tools/sgemm_bench.py > $O/split$sp.jsonl 2> $O/split$sp.err || exit $?
  tail -1 $O/split$sp.jsonl
done
