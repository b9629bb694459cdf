#!/bin/bash
# split-operand GEMM: row panels per tile group (RS_GEMM_GROUP_M_X3S) A/B, two interleaved rounds
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3x; rm -rf $O; mkdir -p $O
for r in 1 2; do for g in 8 4 2 16; do
  echo "## round $r GM=$g" >> $O/gm.txt
  RS_GEMM_GROUP_M_X3S=$g VARIANTS=x3s-f32-prod,x3s-gelu2-prod timeout -k 10 200 python -u tools/x3s_bench.py 131072 2>/dev/null | grep "^M=" | sed 's/err32.*e-07  //' >> $O/gm.txt || exit 1
done; done
cat $O/gm.txt
