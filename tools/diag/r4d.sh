#!/bin/bash
# round 4 GPU session d: cfg-11 trainer GEMM tests and timings, ping-pong / desync probes,
# in-process A/B of the epilogue phase shift (RS_X3S_PHASE)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4d; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_sgemm.py -m gpu -x -q -k "11" --timeout 120 --timeout-method thread > $O/sg11.log 2>&1 || { tail -30 $O/sg11.log; exit 1; }
tail -2 $O/sg11.log
SG_CFGS=0,9,11 timeout -k 10 300 python -u tools/sgemm_bench.py > $O/sgemm.txt 2>&1 || { cat $O/sgemm.txt; exit 1; }
cat $O/sgemm.txt
PROBE=desync SHAPES=2304x768,3072x768 timeout -k 10 300 python -u tools/x3s_epi_probe.py 262144 3 > $O/desync.txt 2>&1 || { cat $O/desync.txt; exit 1; }
cat $O/desync.txt
timeout -k 10 400 python -u tools/env_ab.py 100 3 '' 'RS_X3S_PHASE=33,33,40,0' 'RS_X3S_PHASE=20,20,25,0' 'RS_X3S_PHASE=33,33,40,120' > $O/phase_ab.txt 2>&1 || { cat $O/phase_ab.txt; exit 1; }
cat $O/phase_ab.txt
PROBE=pp SHAPES=2304x768,768x3072 timeout -k 10 300 python -u tools/x3s_epi_probe.py 262144 3 > $O/pp.txt 2>&1 || { cat $O/pp.txt; exit 1; }
cat $O/pp.txt
