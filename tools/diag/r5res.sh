#!/bin/bash
# Round 5: is the LayerNorm epilogue's residual read bound by its HBM burst?  Timing-diagnostic
# builds (wrong results): r0 = residual read from row panel 0 (L2-resident, VAR 536870912),
# r0s0 = that plus the stores onto panel 0 (VAR 33554432) — vs the committed build, per-kind
# bench times interleaved, then the phase stamps of each build.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5res; rm -rf $O; mkdir -p $O
for r in 1 2; do
  for L in head r0 r0s0; do
    export RS_LIBRESCORE=$PWD/ab/librescore_$L.so
    timeout -k 10 300 python -u bench.py --utts 100 --steps 2 --warmup 1 --cpu-seconds 0 --fp16-steps 0 --finetune-steps 0 --c4-secondary 0 > $O/b_${L}_$r.json 2> $O/b_err.log || { tail -20 $O/b_err.log; exit 1; }
    echo "$L round $r: $(python -c "import json;d=json.load(open('$O/b_${L}_$r.json'));print(d['value'], d['kinds_ms'])")"
  done
done
for L in head r0 r0s0; do
  export RS_LIBRESCORE=$PWD/ab/librescore_$L.so
  timeout -k 10 300 python -u tools/stamps.py 50 > $O/stamps_$L.txt 2>&1 || { tail -20 $O/stamps_$L.txt; exit 1; }
  echo "$L: $(grep oproj $O/stamps_$L.txt)"; echo "$L: $(grep ffn2 $O/stamps_$L.txt)"
done
