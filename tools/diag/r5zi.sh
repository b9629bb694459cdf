#!/bin/bash
# Round 5 final tree (VAR 64 uninstantiated; production ISA unchanged): GPU suite + smoke.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5zi; rm -rf $O; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1; rc=$?
echo "suite rc=$rc"; tail -2 $O/gpu_suite.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; tail -1 $O/smoke.log
