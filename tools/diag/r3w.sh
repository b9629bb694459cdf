#!/bin/bash
# split-operand GEMM: half-step stagger of the younger wave half (VAR 524288) vs production,
# interleaved in one process (tools/x3s_bench.py; the stagger is checked bitwise against production)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3w; rm -rf $O; mkdir -p $O
V=x3s-f32-prod,x3s16-f32-pfA,x3s-gelu2-prod,x3s16-gelu2-pfA,x3s16-f32-noepi,x3s16-f32-pfA-noepi
VARIANTS=$V timeout -k 10 400 python -u tools/x3s_bench.py 131072 > $O/x3s.txt 2>&1; rc=$?
cat $O/x3s.txt | tail -8; exit $rc
