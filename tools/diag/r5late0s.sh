#!/bin/bash
# Round 5: the fp32 / GELU GEMMs' next-tile stage 0 issued after the first row-block pair's stores
# (VAR 1073741824; K-step 0 then waits vmcnt(24)) instead of in the bias phase — vs the committed
# build: per-kind bench times interleaved, the phase stamps of each build, GEMM / BERT tests.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5late0s; rm -rf $O; mkdir -p $O
for r in 1 2; do
  for L in head late0s; do
    export RS_LIBRESCORE=$PWD/ab/librescore_$L.so
    timeout -k 10 300 python -u bench.py --utts 100 --steps 2 --warmup 1 --cpu-seconds 0 --fp16-steps 0 --finetune-steps 0 --c4-secondary 0 > $O/b_${L}_$r.json 2> $O/b_err.log || { tail -20 $O/b_err.log; exit 1; }
    echo "$L round $r: $(python -c "import json;d=json.load(open('$O/b_${L}_$r.json'));print(d['value'], d['kinds_ms'])")"
  done
done
for L in head late0s; do
  export RS_LIBRESCORE=$PWD/ab/librescore_$L.so
  timeout -k 10 300 python -u tools/stamps.py 50 > $O/stamps_$L.txt 2>&1 || { tail -20 $O/stamps_$L.txt; exit 1; }
  echo "$L: $(grep qkv $O/stamps_$L.txt)"; echo "$L: $(grep ffn1 $O/stamps_$L.txt)"
done
export RS_LIBRESCORE=$PWD/ab/librescore_late0s.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_bert.py tests/test_gpu_gemm.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_late0s.log 2>&1; rc=$?
echo "late0s tests rc=$rc: $(tail -1 $O/pytest_late0s.log)"
