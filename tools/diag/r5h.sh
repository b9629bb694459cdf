#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5h; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_robust.py -m gpu -v -s --timeout 120 --timeout-method thread > $O/robust.log 2>&1; echo "robust rc=$?"; grep -E "PASS|FAIL|RS_EHIP after|scored on|passed|failed|^E " $O/robust.log | tail -20
