#!/bin/bash
# Round 5: split-operand probe (where the K loop's staging time goes: nowait / alias / noepi) and
# the launch-chunk size (bench --max-rows 261120 vs 522240), interleaved.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5v; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u tools/x3s_epi_probe.py 262144 5 > $O/epi.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/epi.txt
for r in 1 2; do
  for m in 262144 524288; do
    timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-seconds 0 --fp16-steps 0 --finetune-steps 0 --c4-secondary 0 --no-profile --max-rows $m > $O/b_${m}_$r.json 2> $O/b_${m}_$r.err || { tail -5 $O/b_${m}_$r.err; exit 1; }
    echo "max_rows $m round $r: $(python -c "import json;d=json.load(open('$O/b_${m}_$r.json'));print(d['value'], d['kinds_ms'])")"
  done
done
