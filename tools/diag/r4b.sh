#!/bin/bash
# round 4 GPU session b: robustness + pp tests, epilogue probe (incl. the ping-pong kernel),
# end-to-end A/B (RS_PP, RS_CHUNK_ALIGN), LM fine-tune probe
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4b; rm -rf $O; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_robust.py tests/test_gpu_gemm.py tests/test_gpu_bert.py -k "robust or pp or lnfuse_scores or rccl or deferred or chunks or xcd or timeout" -x -v --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -25 $O/tests.log
timeout -k 10 300 python -u tools/x3s_epi_probe.py 262144 2 > $O/epi.txt 2>&1 || { cat $O/epi.txt; exit 1; }
cat $O/epi.txt
for r in 1 2; do
  for cfg in "1 0" "1 1" "0 0"; do
    set -- $cfg
    RS_CHUNK_ALIGN=$1 RS_PP=$2 timeout -k 10 200 python -u bench.py --utts 100 --steps 2 --warmup 1 --cpu-seconds 0 --fp16-steps 0 --no-profile --finetune-steps 0 > $O/bench_a$1_p$2_$r.json 2>$O/bench_err.log || { tail -20 $O/bench_err.log; exit 1; }
    echo "align=$1 pp=$2 round $r: $(python -c "import json;d=json.load(open('$O/bench_a$1_p$2_$r.json'));print(d['value'], d['ms_per_step'])")"
  done
done
timeout -k 10 300 python -u tools/diag/r4_finetune_probe.py 200 1e-4 64 0 150 300 600 > $O/ft.txt 2>&1 || { tail -20 $O/ft.txt; exit 1; }
cat $O/ft.txt
