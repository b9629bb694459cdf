#!/bin/bash
# round 6, final tree: the GPU suite, smoke(), the default bench line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6final
rm -rf $O && mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=6 --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
rc=$?
tail -5 $O/gputest.log
echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -3 $O/smoke.log
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err
rc2=$?
tail -c 1500 $O/bench.json
exit $rc2
