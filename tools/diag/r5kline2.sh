#!/bin/bash
# Round 5: the full-line K-loop DMA diagnostic (VAR 4096) split by operand: W side only (+16) and
# A side only (+32) — per-kind bench times interleaved with the committed build, then phase stamps.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5kline2; rm -rf $O; mkdir -p $O
for r in 1; do
  for L in head wonly aonly; do
    export RS_LIBRESCORE=$PWD/ab/librescore_$L.so
    timeout -k 10 300 python -u bench.py --utts 100 --steps 2 --warmup 1 --cpu-seconds 0 --fp16-steps 0 --finetune-steps 0 --c4-secondary 0 > $O/b_${L}_$r.json 2> $O/b_err.log || { tail -20 $O/b_err.log; exit 1; }
    echo "$L round $r: $(python -c "import json;d=json.load(open('$O/b_${L}_$r.json'));print(d['value'], d['kinds_ms'])")"
  done
done
for L in head wonly aonly; do
  export RS_LIBRESCORE=$PWD/ab/librescore_$L.so
  timeout -k 10 300 python -u tools/stamps.py 50 > $O/stamps_$L.txt 2>&1 || { tail -20 $O/stamps_$L.txt; exit 1; }
  grep -E "qkv|oproj|ffn1|ffn2" $O/stamps_$L.txt | sed "s/^/$L: /"
done
