#!/bin/bash
# round 4 GPU session k: launch-chunk size A/B (max_rows 262144 vs 524288 vs 1048576), interleaved
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4k; rm -rf $O; mkdir -p $O
for r in 1 2; do
  for mr in 262144 524288 1048576; do
    timeout -k 10 300 python -u bench.py --max-rows $mr --steps 2 --warmup 1 --cpu-seconds 0 --fp16-steps 0 --no-profile --finetune-steps 0 > $O/b_${mr}_$r.json 2> $O/err.log || { tail -20 $O/err.log; exit 1; }
    echo "max_rows=$mr round $r: $(python -c "import json;d=json.load(open('$O/b_${mr}_$r.json'));print(d['value'], d['ms_per_step'])")"
  done
done
