#!/bin/bash
# round 4 GPU session c: where the ping-pong kernel loses (variants of k_gemm_pp.hip)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4c; rm -rf $O; mkdir -p $O
PROBE=pp SHAPES=2304x768,768x3072 timeout -k 10 300 python -u tools/x3s_epi_probe.py 262144 3 > $O/pp.txt 2>&1 || { cat $O/pp.txt; exit 1; }
cat $O/pp.txt
PROBE=desync SHAPES=2304x768,3072x768 timeout -k 10 300 python -u tools/x3s_epi_probe.py 262144 3 > $O/desync.txt 2>&1 || { cat $O/desync.txt; exit 1; }
cat $O/desync.txt
