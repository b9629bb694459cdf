#!/bin/bash
# round 5 GPU session b: in-process A/B of RS_LNKRES x RS_LNGANG, and the new build against the
# round-4 build (ab/librescore_r4.so)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5b; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u tools/env_ab.py 100 3 'RS_LNKRES=0' 'RS_LNKRES=1' 'RS_LNKRES=2' 'RS_LNKRES=1;RS_LNGANG=xcd' 'RS_LNKRES=0;RS_LNGANG=xcd' > $O/env_ab.txt 2>&1 || { tail -20 $O/env_ab.txt; exit 1; }
cat $O/env_ab.txt
for r in 1 2; do
  for L in r4 new; do
    if [ $L = r4 ]; then export RS_LIBRESCORE=$PWD/ab/librescore_r4.so; else unset RS_LIBRESCORE; fi
    timeout -k 10 300 python -u bench.py --utts 100 --steps 2 --warmup 1 --cpu-seconds 0 --fp16-steps 0 --finetune-steps 0 --c4-secondary 0 > $O/b_${L}_$r.json 2> $O/b_err.log || { tail -20 $O/b_err.log; exit 1; }
    echo "$L round $r: $(python -c "import json;d=json.load(open('$O/b_${L}_$r.json'));print(d['value'], d['kinds_ms'])")"
  done
done
