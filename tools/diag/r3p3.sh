#!/bin/bash
# fused LayerNorm epilogue: next tile stage-0 DMA issued after the residual loads (default) vs before (RS_LNDMA_EARLY=1)
# parity of the LayerNorm-epilogue paths, then interleaved A/B against the default
set -o pipefail
O=gpurun_out/r3p3; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_bert.py tests/test_gpu_configs.py -x -q --timeout 240 --timeout-method thread -k "lnfuse or fp16x3 or dedup or range_guard or c3_shape or c4_shape" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --utts 100 --steps 2 --warmup 1 --cpu-seconds 0 --fp16-steps 0 > $O/$tag.json 2> $O/$tag.err || { tail -20 $O/$tag.err; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag', d['value'], d['kinds_ms'])"
}
for r in 1 2; do
  run early_r$r RS_LNDMA_EARLY=1 || exit 1
  run late_r$r RS_LNDMA_EARLY=0 || exit 1
done
