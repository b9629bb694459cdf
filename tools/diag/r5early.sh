#!/bin/bash
# Round 5: the LayerNorm GEMM's first residual batch issued right behind the bias loads (VAR 2097152;
# the bias wait becomes vmcnt(8)) so its round trip runs under the bias wait and the transition —
# vs the committed build: per-kind bench times interleaved, phase stamps, BERT / GEMM parity tests.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5early; rm -rf $O; mkdir -p $O
for r in 1 2; do
  for L in head early; do
    export RS_LIBRESCORE=$PWD/ab/librescore_$L.so
    timeout -k 10 300 python -u bench.py --utts 100 --steps 2 --warmup 1 --cpu-seconds 0 --fp16-steps 0 --finetune-steps 0 --c4-secondary 0 > $O/b_${L}_$r.json 2> $O/b_err.log || { tail -20 $O/b_err.log; exit 1; }
    echo "$L round $r: $(python -c "import json;d=json.load(open('$O/b_${L}_$r.json'));print(d['value'], d['kinds_ms'])")"
  done
done
for L in head early; do
  export RS_LIBRESCORE=$PWD/ab/librescore_$L.so
  timeout -k 10 300 python -u tools/stamps.py 50 > $O/stamps_$L.txt 2>&1 || { tail -20 $O/stamps_$L.txt; exit 1; }
  echo "$L: $(grep oproj $O/stamps_$L.txt)"; echo "$L: $(grep ffn2 $O/stamps_$L.txt)"
done
export RS_LIBRESCORE=$PWD/ab/librescore_early.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_bert.py tests/test_gpu_gemm.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_early.log 2>&1; rc=$?
echo "early tests rc=$rc: $(tail -1 $O/pytest_early.log)"
