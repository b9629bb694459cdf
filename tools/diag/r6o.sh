#!/bin/bash
# Round 6: the LayerNorm epilogue's residual by whole-line LDS-DMA (RS_LNRES_DMA=1, VAR 4) —
# robustness / BERT tests under it, bitwise vs the register-load form, interleaved bench A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6o; rm -rf $O; mkdir -p $O
L=asr-rescoring_amd/librescore.so
RS_LNRES_DMA=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_robust.py tests/test_gpu_bert.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 600 python -u tools/bitwise_ab.py $L $L@RS_LNRES_DMA=1 $O > $O/bitwise.json 2> $O/bitwise.err && \
for d in 1 0 1 0; do
  RS_LNRES_DMA=$d timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-seconds 0 --fp16-steps 0 --c4-secondary 0 --finetune-steps 0 >> $O/bench_ab.jsonl 2>> $O/bench_ab.err || exit 1
done
rc=$?
tail -n 3 $O/tests.log; cat $O/bitwise.json; python -c "
import json
for l in open('$O/bench_ab.jsonl'):
    r=json.loads(l); print(r['value'], r['kinds_ms'])
"
exit $rc
