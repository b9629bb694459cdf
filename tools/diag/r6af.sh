#!/bin/bash
# round 6: after retiring the dominated trainer GEMM configurations — parity, sweep
set -o pipefail
O=gpurun_out/r6af
rm -rf $O && mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_sgemm.py tests/test_gpu_train.py > $O/tests.txt 2>&1
rc=$?
tail -3 $O/tests.txt
[ $rc -eq 0 ] || exit $rc
SG_CFGS=11,12,17 timeout -k 10 300 python -u tools/sgemm_bench.py > $O/sgemm_all.jsonl 2> $O/sgemm_bench.err || exit $?
tail -1 $O/sgemm_all.jsonl
