#!/bin/bash
# Round 5: cross-process occupier robustness tests on the cancellable XCD-local gang build, then an
# interleaved xcd/ticket throughput A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5i; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_robust.py -m gpu -v -s --timeout 120 --timeout-method thread > $O/robust.log 2>&1; rc=$?; echo "robust rc=$rc"; grep -E "PASS|FAIL|RS_EHIP after|scored on|passed|failed|^E " $O/robust.log | tail -24
[ $rc -eq 0 -o $rc -eq 1 ] || exit $rc
timeout -k 10 400 python -u tools/env_ab.py 100 4 '' 'RS_LNGANG=ticket' > $O/ab.txt 2>&1; echo "ab rc=$?"; grep -v amdgpu.ids $O/ab.txt | tail -8
