#!/bin/bash
# round 4 GPU session f: trainer GEMM cfg 11 (64x64 direct-to-register) tests + timings
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4f; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_sgemm.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/sgtests.log 2>&1 || { tail -30 $O/sgtests.log; exit 1; }
tail -2 $O/sgtests.log
SG_CFGS=0,9,11 timeout -k 10 300 python -u tools/sgemm_bench.py > $O/sgemm.txt 2>&1 || { cat $O/sgemm.txt; exit 1; }
cat $O/sgemm.txt
