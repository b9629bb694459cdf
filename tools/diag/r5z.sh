#!/bin/bash
# Round 5: LayerNorm-epilogue residual batches two deep (ab/librescore_rp.so = working tree) vs the
# committed build (ab/librescore_head.so): LayerNorm / robustness tests on the new build, interleaved A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5z; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_bert.py tests/test_gpu_robust.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in head rp; do
    RS_LIBRESCORE=ab/librescore_$v.so timeout -k 10 300 python -u tools/env_ab.py 100 3 '' > $O/${v}_$r.txt 2>&1 || exit 1
    echo "$v $r: $(grep -E 'masked fwd/s' $O/${v}_$r.txt | tail -1)"
  done
done
