#!/bin/bash
# Round 5: static panel lists with cancellable gangs (ab/librescore_static.so) and panel lists taken
# from a list counter (ab/librescore_list.so = the working tree) vs the committed build; robustness
# tests on the list build.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5q; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_robust.py -m gpu -v -s --timeout 120 --timeout-method thread > $O/robust.log 2>&1; rc=$?
echo "robust rc=$rc"; grep -E "scored|passed|failed|^E " $O/robust.log | tail -12
[ $rc -eq 0 -o $rc -eq 1 ] || exit $rc
for r in 1 2 3; do
  for v in head static list; do
    RS_LIBRESCORE=ab/librescore_$v.so timeout -k 10 300 python -u tools/env_ab.py 100 3 '' > $O/${v}_$r.txt 2>&1 || exit 1
    echo "$v $r: $(grep -E 'masked fwd/s' $O/${v}_$r.txt | tail -1)"
  done
done
