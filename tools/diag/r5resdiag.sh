#!/bin/bash
# Round 5: what the LayerNorm GEMM's residual phase waits on.  Timing-diagnostic builds (wrong
# results): nold = the residual taken as 0 without its loads (VAR 2097152 in that build; the bit now
# selects the full-line form of tools/diag/r5resline.sh), noadd = the residual add skipped
# (VAR 8388608) — phase stamps of each build beside the committed build.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5resdiag; rm -rf $O; mkdir -p $O
for L in head nold noadd; do
  export RS_LIBRESCORE=$PWD/ab/librescore_$L.so
  timeout -k 10 300 python -u tools/stamps.py 50 > $O/stamps_$L.txt 2>&1 || { tail -20 $O/stamps_$L.txt; exit 1; }
  echo "$L: $(grep oproj $O/stamps_$L.txt)"; echo "$L: $(grep ffn2 $O/stamps_$L.txt)"
done
