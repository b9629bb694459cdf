#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5g; rm -rf $O; mkdir -p $O
timeout -k 10 200 python -u tools/diag/occupy_probe.py > $O/occupy.txt 2>&1; echo rc=$?; grep -v amdgpu.ids $O/occupy.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_robust.py -m gpu -v -s --timeout 120 --timeout-method thread -k "two_streams or too_few or three_free" > $O/robust.log 2>&1; echo "robust rc=$?"; grep -E "PASS|FAIL|RS_EHIP after|passed|failed|^E " $O/robust.log | tail -12
