#!/bin/bash
# round 5 GPU session s (final kernel): the GPU suite, the default bench line (with c4_secondary), a rocprofv3
# kernel trace of the headline steps, smoke
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5s; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1; rc=$?
echo "suite rc=$rc"; grep -E "FAIL|passed|failed" $O/gpu_suite.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench.json'))
print('value', d['value'], 'ms/step', d['ms_per_step'], 'frac', d['roofline']['frac'], 'kinds', d['kinds_ms'])
print('c4', json.dumps(d['c4_secondary']))
print('cpu', json.dumps(d['cpu_baseline'])[:400])
print('rerank', d['rerank'])
"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --fp16-steps 0 --c4-secondary 0 > $O/bench_under_rocprof.json 2> $O/kt.err || { tail -20 $O/kt.err; exit 1; }
cp "$(find $O/kt -name '*kernel_stats.csv' | head -1)" $O/kernel_stats.csv
head -12 $O/kernel_stats.csv | cut -c1-200
rm -rf $O/kt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; tail -2 $O/smoke.log
