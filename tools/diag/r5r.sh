#!/bin/bash
# Round 5: split-operand GEMM row-panel group size (RS_GEMM_GROUP_M_X3S, read once per process) —
# throughput, interleaved in separate processes, then FETCH_SIZE per kernel for 8 vs the best other.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5r; rm -rf $O; mkdir -p $O
for r in 1 2; do
  for g in 8 4 16 2; do
    RS_GEMM_GROUP_M_X3S=$g timeout -k 10 300 python -u tools/env_ab.py 100 3 '' > $O/gm${g}_$r.txt 2>&1 || exit 1
    echo "gm $g round $r: $(grep -E 'masked fwd/s' $O/gm${g}_$r.txt | tail -1)"
  done
done
for g in 8 4 16; do
  RS_GEMM_GROUP_M_X3S=$g timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$g -o run -- python -u tools/env_ab.py 30 1 '' > /dev/null 2>&1 || exit 1
  RS_GEMM_GROUP_M_X3S=$g timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pf_$g -o run -- python -u tools/env_ab.py 30 1 '' > /dev/null 2>&1 || exit 1
  echo "== gm $g"; python tools/diag/kt_summary.py $O/kt_$g $O/pf_$g | tee $O/summary_gm$g.txt
done
rm -rf $O/kt_* $O/pf_*
