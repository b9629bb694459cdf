#!/bin/bash
# Round 5: the GELU image with the permuted-column layout (16-B slab writes) — the GPU
# suite on the new build, then an interleaved A/B vs the committed build (ab/librescore_head.so).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5perm; rm -rf $O; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1; rc=$?
echo "suite rc=$rc"; tail -3 $O/gpu_suite.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in head perm; do
    RS_LIBRESCORE=ab/librescore_$v.so timeout -k 10 300 python -u tools/env_ab.py 100 3 '' > $O/${v}_$r.txt 2>&1 || exit 1
    echo "$v $r: $(grep -E 'masked fwd/s' $O/${v}_$r.txt | tail -1)"
  done
done
