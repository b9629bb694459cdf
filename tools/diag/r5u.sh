#!/bin/bash
# Round 5: one in-register operand scaling per K-step (64 W_hi; accumulators at 64 C, ab/librescore_up.so)
# — GPU suite and K-loop scaling probe on it; interleaved A/B vs the gang-list build (list) and the
# branch-free K-loop DMA build (nobr, spills 10-19 VGPRs in the fp32 / GELU instances).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5u; rm -rf $O; mkdir -p $O
RS_LIBRESCORE=ab/librescore_up.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1; rc=$?
echo "suite rc=$rc"; tail -4 $O/gpu_suite.log
[ $rc -eq 0 ] || exit $rc
RS_LIBRESCORE=ab/librescore_up.so PROBE=scale timeout -k 10 300 python -u tools/x3s_epi_probe.py 262144 5 > $O/scale.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/scale.txt
for r in 1 2 3; do
  for v in list up nobr; do
    RS_LIBRESCORE=ab/librescore_$v.so timeout -k 10 300 python -u tools/env_ab.py 100 3 '' > $O/${v}_$r.txt 2>&1 || exit 1
    echo "$v $r: $(grep -E 'masked fwd/s' $O/${v}_$r.txt | tail -1)"
  done
done
