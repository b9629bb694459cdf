#!/bin/bash
# GPU parity suite + a bench line (GPU box, repo root): bash tools/gpu_tests.sh <tag> [pytest selectors...]
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG
rm -rf $O && mkdir -p $O
SEL=${@:-tests}
timeout -k 10 1000 python -u -m pytest $SEL -m gpu -v --maxfail=6 --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
rc=$?
tail -40 $O/gputest.log
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 > $O/bench.json 2> $O/bench.err
rc2=$?
tail -c 2500 $O/bench.json
exit $rc2
