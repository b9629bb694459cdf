#!/bin/bash
# round 6: where the trainer GEMM's K-step goes at one workgroup per CU — MFMA busy and clock of
# cfg 0 / 12 / 13 / 14 against torch's fp32 matmul on 5300 x 768 x 3072 (fwd, dgrad)
set -eo pipefail
export TMPDIR=/tmp
O=gpurun_out/r6w
rm -rf $O && mkdir -p $O
export SG_CFGS=0,12,13,14 REPS=20
for f in fwd dgrad; do
  timeout -k 10 120 python -u tools/sgemm_one.py 5300 768 3072 $f >> $O/times.txt 2>> $O/err.txt
  timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_$f -o run --output-format csv -- \
      python tools/sgemm_one.py 5300 768 3072 $f > /dev/null 2>> $O/err.txt
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt_$f -o run --output-format csv -- \
      python tools/sgemm_one.py 5300 768 3072 $f > /dev/null 2>> $O/err.txt
done
cat $O/times.txt
