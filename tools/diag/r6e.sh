#!/bin/bash
# Round 6: GELU in a = |x| (folded coefficients) + fma-form lo split — GELU accuracy test, the GEMM and
# fp16x3 parity tests, and an interleaved bench A/B against the previous build (ab/r6a).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6e; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_bert.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 && \
for lib in asr-rescoring_amd/librescore.so ab/r6a/librescore.so asr-rescoring_amd/librescore.so ab/r6a/librescore.so; do
  RS_LIBRESCORE=$lib timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-seconds 0 --fp16-steps 0 --c4-secondary 0 --finetune-steps 0 >> $O/bench_ab.jsonl 2>> $O/bench_ab.err || exit 1
done
rc=$?
tail -n 3 $O/tests.log; python -c "
import json
for l in open('$O/bench_ab.jsonl'):
    r=json.loads(l); print(r['value'], r['kinds_ms'])
"
exit $rc
