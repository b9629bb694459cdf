#!/bin/bash
# round 6: software-pipelined trainer GEMM (cfg 12-14) — parity on every form, then the shape sweep
set -o pipefail
O=gpurun_out/r6v
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sgemm.py > $O/sgemm_tests.txt 2>&1
rc=$?
tail -3 $O/sgemm_tests.txt
[ $rc -eq 0 ] || exit $rc
SG_CFGS=0,9,11,12,13,14 timeout -k 10 400 python -u tools/sgemm_bench.py > $O/sgemm_all.jsonl 2> $O/sgemm_bench.err
rc=$?
tail -2 $O/sgemm_all.jsonl
exit $rc
