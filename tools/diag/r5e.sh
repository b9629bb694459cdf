#!/bin/bash
# round 5 GPU session e: trainer GEMM, every tile configuration on every training shape vs rocBLAS
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5e; rm -rf $O; mkdir -p $O
SG_CFGS=0,1,2,3,4,5,6,7,8,9,10,11 timeout -k 10 600 python -u tools/sgemm_bench.py > $O/sgemm_all.jsonl 2> $O/err.log || { tail -20 $O/err.log; exit 1; }
tail -3 $O/sgemm_all.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_robust.py tests/test_gpu_bert.py -m gpu -v -s --timeout 120 --timeout-method thread > $O/robust.log 2>&1
echo "robust rc=$?"; grep -E "FAIL|RS_EHIP after|passed|failed" $O/robust.log | tail -12
