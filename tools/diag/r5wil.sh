#!/bin/bash
# Round 5: the W image interleaved [hi 32 | lo 32] per K-step (x3s VAR 64; ran through an rs_debug_gemm dbg 64
# entry and tools/x3s_epi_probe.py PROBE=wil, both since removed): bitwise check and isolated timing.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5wil; rm -rf $O; mkdir -p $O
PROBE=wil timeout -k 10 400 python -u tools/x3s_epi_probe.py 262144 3 > $O/probe.txt 2>&1; rc=$?
cat $O/probe.txt; exit $rc
