#!/bin/bash
# Round 5: the LayerNorm GEMM's residual loads at full-line granularity (VAR 2097152, timing
# diagnostic, wrong results: each load covers 8 rows x 128 B instead of 16 rows x 64 B — the same
# rows, bytes and lines) — phase stamps beside the committed build.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5resline; rm -rf $O; mkdir -p $O
for L in head line; do
  export RS_LIBRESCORE=$PWD/ab/librescore_$L.so
  timeout -k 10 300 python -u tools/stamps.py 50 > $O/stamps_$L.txt 2>&1 || { tail -20 $O/stamps_$L.txt; exit 1; }
  echo "$L: $(grep oproj $O/stamps_$L.txt)"; echo "$L: $(grep ffn2 $O/stamps_$L.txt)"
done
