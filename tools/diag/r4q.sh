#!/bin/bash
# round 4 GPU session q: epilogue store policy (probe) and alternating panel directions (end to end)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4q; rm -rf $O; mkdir -p $O
PROBE=spol SHAPES=2304x768,3072x768,768x3072 timeout -k 10 300 python -u tools/x3s_epi_probe.py 262144 5 > $O/spol.txt 2>&1 || { cat $O/spol.txt; exit 1; }
cat $O/spol.txt
timeout -k 10 500 python -u tools/env_ab.py 200 3 '' 'RS_ALT_DIR=1' > $O/altdir.txt 2>&1 || { cat $O/altdir.txt; exit 1; }
cat $O/altdir.txt
