#!/bin/bash
# Round 5: LayerNorm gangs that claim their row panels — robustness tests beside another process,
# the GPU suite, then an interleaved end-to-end A/B against the committed build (ab/librescore_head.so).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5l; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_robust.py -m gpu -v -s --timeout 120 --timeout-method thread > $O/robust.log 2>&1; rc=$?
echo "robust rc=$rc"; grep -E "PASS|FAIL|scored|passed|failed|^E " $O/robust.log | tail -24
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1; rc=$?
echo "suite rc=$rc"; tail -5 $O/gpu_suite.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in head new; do
    if [ $v = head ]; then L=ab/librescore_head.so; else L=asr-rescoring_amd/librescore.so; fi
    RS_LIBRESCORE=$L timeout -k 10 300 python -u tools/env_ab.py 100 3 '' > $O/ab_${v}_${r}.txt 2>&1 || exit 1
    echo "$v $r: $(grep -E 'masked fwd/s' $O/ab_${v}_${r}.txt | tail -1)"
  done
done
