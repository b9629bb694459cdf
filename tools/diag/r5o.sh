#!/bin/bash
# Round 5: which kernels the claimed-panel build slows — kernel trace + FETCH_SIZE, committed build vs new.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5o; rm -rf $O; mkdir -p $O
for v in head new; do
  if [ $v = head ]; then L=ab/librescore_head.so; else L=asr-rescoring_amd/librescore.so; fi
  RS_LIBRESCORE=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o run -- python -u tools/env_ab.py 100 2 '' > $O/kt_$v.txt 2>&1 || { tail -5 $O/kt_$v.txt; exit 1; }
  RS_LIBRESCORE=$L timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pf_$v -o run -- python -u tools/env_ab.py 30 1 '' > $O/pf_$v.txt 2>&1 || { tail -5 $O/pf_$v.txt; exit 1; }
  echo "== $v"; python tools/diag/kt_summary.py $O/kt_$v $O/pf_$v | tee $O/summary_$v.txt
done
rm -rf $O/kt_* $O/pf_*
