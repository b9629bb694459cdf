#!/bin/bash
# fused residual + LayerNorm: cost of the in-launch statistics exchange (RS_LNFUSE_DIAG=1: own
# partials only, wrong LN, timing only) and of the residual read (DIAG=4), vs the separate pass
set -o pipefail
O=gpurun_out/r3z; rm -rf $O; mkdir -p $O
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --utts 100 --steps 2 --warmup 1 --cpu-seconds 0 --fp16-steps 0 > $O/$tag.json 2> $O/$tag.err || { tail -20 $O/$tag.err; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag', d['value'], d['kinds_ms'])"
}
for r in 1 2; do
  run on_r$r RS_LNFUSE=1 || exit 1
  run noxchg_r$r RS_LNFUSE=1 RS_LNFUSE_DIAG=1 || exit 1
  run hitres_r$r RS_LNFUSE=1 RS_LNFUSE_DIAG=4 || exit 1
  run off_r$r RS_LNFUSE=0 || exit 1
done
