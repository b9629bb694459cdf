#!/bin/bash
# Round 5 final tree (per-operand diagnostic bits; production kernels unchanged): GPU suite, the
# default bench line, smoke.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5zh; rm -rf $O; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1; rc=$?
echo "suite rc=$rc"; tail -2 $O/gpu_suite.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench.json'))
print('value', d['value'], 'ms/step', d['ms_per_step'], 'frac', d['roofline']['frac'], 'kinds', d['kinds_ms'])
"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; tail -1 $O/smoke.log
