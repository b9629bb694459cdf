#!/bin/bash
# round 4 first GPU session: robustness tests, epilogue probe, fine-tune probe, chunk-align A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4a; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_robust.py -x -v --timeout 150 --timeout-method thread > $O/robust.log 2>&1 || { tail -40 $O/robust.log; exit 1; }
tail -12 $O/robust.log
timeout -k 10 300 python -u tools/x3s_epi_probe.py 262144 3 > $O/epi.txt 2>&1 || { cat $O/epi.txt; exit 1; }
cat $O/epi.txt
timeout -k 10 300 python -u tools/diag/r4_finetune_probe.py 200 1e-4 64 0 150 300 600 > $O/ft.txt 2>&1 || { tail -20 $O/ft.txt; exit 1; }
cat $O/ft.txt
for r in 1 2; do
  for a in 0 1; do
    RS_CHUNK_ALIGN=$a timeout -k 10 200 python -u bench.py --utts 100 --steps 2 --warmup 1 --cpu-seconds 0 --fp16-steps 0 --no-profile > $O/bench_align${a}_$r.json 2>$O/bench_err.log || { tail -20 $O/bench_err.log; exit 1; }
    echo "align=$a round $r: $(python -c "import json,sys;d=json.load(open('$O/bench_align${a}_$r.json'));print(d['value'], d['ms_per_step'])")"
  done
done
