#!/bin/bash
# Round 5: claimed panels handed over three tiles ahead — robustness tests + interleaved A/B vs the committed build.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5n; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_robust.py -m gpu -v -s --timeout 120 --timeout-method thread > $O/robust.log 2>&1; rc=$?
echo "robust rc=$rc"; grep -E "scored|passed|failed|^E " $O/robust.log | tail -12
[ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in head new; do
    if [ $v = head ]; then L=ab/librescore_head.so; else L=asr-rescoring_amd/librescore.so; fi
    RS_LIBRESCORE=$L timeout -k 10 300 python -u tools/env_ab.py 100 3 '' > $O/ab_${v}_${r}.txt 2>&1 || exit 1
    echo "$v $r: $(grep -E 'masked fwd/s' $O/ab_${v}_${r}.txt | tail -1)"
  done
done
