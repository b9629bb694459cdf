# fused residual + LayerNorm epilogue: where its cost goes (interleaved A/B, timing diagnostics)
set -o pipefail
O=gpurun_out/r3j; mkdir -p $O
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --utts 100 --steps 2 --warmup 1 --cpu-seconds 0 --fp16-steps 0 --no-profile > $O/$tag.json 2> $O/$tag.err || { tail -20 $O/$tag.err; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag', d['value'])"
}
for r in 1 2; do
  run off_r$r RS_LNFUSE=0 || exit 1
  run on_r$r RS_LNFUSE=1 || exit 1
  run nowait_r$r RS_LNFUSE=1 RS_LNFUSE_DIAG=1 || exit 1
  run sleep16_r$r RS_LNFUSE=1 RS_LNFUSE_DIAG=2 || exit 1
  run nores_r$r RS_LNFUSE=1 RS_LNFUSE_DIAG=4 || exit 1
  run nowait_nores_r$r RS_LNFUSE=1 RS_LNFUSE_DIAG=5 || exit 1
done
# per-kind times of one profiled run each
for f in 0 1; do
  RS_LNFUSE=$f timeout -k 10 300 python -u bench.py --utts 100 --steps 2 --warmup 1 --cpu-seconds 0 --fp16-steps 0 > $O/prof_f$f.json 2> $O/prof_f$f.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/prof_f$f.json').read().strip().splitlines()[-1]); print('prof lnfuse=$f', d['value'], d['kinds_ms'])"
done
