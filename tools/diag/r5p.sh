#!/bin/bash
# Round 5: is the claimed-panel build's loss the dynamic order?  new build, claimed vs static order
# (RS_LNFUSE_DIAG=16, experiment), interleaved in one process; the committed build beside it.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5p; rm -rf $O; mkdir -p $O
for r in 1 2; do
  RS_LIBRESCORE=ab/librescore_head.so timeout -k 10 300 python -u tools/env_ab.py 100 3 '' > $O/head_$r.txt 2>&1 || exit 1
  echo "head $r: $(grep -E 'masked fwd/s' $O/head_$r.txt | tail -1)"
  timeout -k 10 300 python -u tools/env_ab.py 100 3 '' 'RS_LNFUSE_DIAG=16' > $O/new_$r.txt 2>&1 || exit 1
  grep -E 'masked fwd/s' $O/new_$r.txt | tail -2
done
