#!/bin/bash
# Round 6: attention ctx image stored as 16-B pieces (v_permlane16_swap) — attention / BERT tests,
# bitwise vs the previous build (ab/g2), interleaved bench A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6g; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_bert.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 600 python -u tools/bitwise_ab.py ab/g2/librescore.so asr-rescoring_amd/librescore.so $O > $O/bitwise.json 2> $O/bitwise.err && \
for lib in asr-rescoring_amd/librescore.so ab/g2/librescore.so asr-rescoring_amd/librescore.so ab/g2/librescore.so; do
  RS_LIBRESCORE=$lib timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-seconds 0 --fp16-steps 0 --c4-secondary 0 --finetune-steps 0 >> $O/bench_ab.jsonl 2>> $O/bench_ab.err || exit 1
done
rc=$?
tail -n 3 $O/tests.log; cat $O/bitwise.json; python -c "
import json
for l in open('$O/bench_ab.jsonl'):
    r=json.loads(l); print(r['value'], r['kinds_ms'])
"
exit $rc
