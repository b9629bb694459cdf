# fused residual + LayerNorm epilogue: parity tests, then an interleaved A/B of the C3 bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3i; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_bert.py -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for r in 1 2; do
  for f in 1 0; do
    RS_LNFUSE=$f timeout -k 10 300 python -u bench.py --utts 100 --steps 3 --warmup 1 --cpu-seconds 0 --fp16-steps 0 > $O/ab_f${f}_r$r.json 2> $O/ab_f${f}_r$r.err || { tail -20 $O/ab_f${f}_r$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/ab_f${f}_r$r.json').read().strip().splitlines()[-1]); print('lnfuse=$f', d['value'], d.get('kinds_ms'), d.get('pll_max_rel_err_vs_oracle', d.get('pll_max_rel_err_vs_gpu')))"
  done
done
