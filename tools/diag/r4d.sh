#!/bin/bash
# round 4 GPU session d: cfg-11 trainer GEMM tests, full GPU suite + smoke + default bench line, then the pp / desync probes
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4d; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_sgemm.py -m gpu -x -q -k "11" --timeout 120 --timeout-method thread > $O/sg11.log 2>&1 || { tail -30 $O/sg11.log; exit 1; }
tail -2 $O/sg11.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
rc=$?; tail -5 $O/gputest.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $O/gputest.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 3000 $O/bench.json
PROBE=pp SHAPES=2304x768,768x3072 timeout -k 10 300 python -u tools/x3s_epi_probe.py 262144 3 > $O/pp.txt 2>&1 || { cat $O/pp.txt; exit 1; }
cat $O/pp.txt
PROBE=desync SHAPES=2304x768,3072x768 timeout -k 10 300 python -u tools/x3s_epi_probe.py 262144 3 > $O/desync.txt 2>&1 || { cat $O/desync.txt; exit 1; }
cat $O/desync.txt
SG_CFGS=0,9,11 timeout -k 10 300 python -u tools/sgemm_bench.py > $O/sgemm.txt 2>&1 || { cat $O/sgemm.txt; exit 1; }
cat $O/sgemm.txt
