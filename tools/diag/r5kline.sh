#!/bin/bash
# Round 5: is the split-operand K loop bound by its per-CU request rate?  Timing-diagnostic build
# (wrong results): every DMA piece covers 8 rows x 128 B instead of 16 rows x 64 B (VAR 4096 in
# all three production instances; the same rows and bytes per K loop) — per-kind bench times
# interleaved with the committed build, then the phase stamps of both.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5kline; rm -rf $O; mkdir -p $O
for r in 1 2; do
  for L in head kline; do
    export RS_LIBRESCORE=$PWD/ab/librescore_$L.so
    timeout -k 10 300 python -u bench.py --utts 100 --steps 2 --warmup 1 --cpu-seconds 0 --fp16-steps 0 --finetune-steps 0 --c4-secondary 0 > $O/b_${L}_$r.json 2> $O/b_err.log || { tail -20 $O/b_err.log; exit 1; }
    echo "$L round $r: $(python -c "import json;d=json.load(open('$O/b_${L}_$r.json'));print(d['value'], d['kinds_ms'])")"
  done
done
for L in head kline; do
  export RS_LIBRESCORE=$PWD/ab/librescore_$L.so
  timeout -k 10 300 python -u tools/stamps.py 50 > $O/stamps_$L.txt 2>&1 || { tail -20 $O/stamps_$L.txt; exit 1; }
  grep -E "qkv|oproj|ffn1|ffn2" $O/stamps_$L.txt | sed "s/^/$L: /"
done
