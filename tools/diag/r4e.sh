#!/bin/bash
# round 4 GPU session e: full GPU suite + smoke + default bench line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4e; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
rc=$?; tail -5 $O/gputest.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $O/gputest.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 3000 $O/bench.json
