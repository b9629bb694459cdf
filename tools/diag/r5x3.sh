#!/bin/bash
# Round 5: 64x-split images — second-half fragment reads pipelined into the first half (x2p, the
# working tree) vs the half-boundary barrier (x2) vs the committed build (head): GEMM / encoder tests on
# x2p, interleaved A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5x3; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_bert.py tests/test_gpu_robust.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in head x2 x2p; do
    RS_LIBRESCORE=ab/librescore_$v.so timeout -k 10 300 python -u tools/env_ab.py 100 3 '' > $O/${v}_$r.txt 2>&1 || exit 1
    echo "$v $r: $(grep -E 'masked fwd/s' $O/${v}_$r.txt | tail -1)"
  done
done
