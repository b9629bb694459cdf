#!/bin/bash
# Round 5 final tree (late stage 0 in the LayerNorm GEMM): the GPU suite, then the r5w measurements
# (default bench line, rocprofv3 kernel stats, PMC traffic + MFMA busy, smoke).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5f2; rm -rf $O; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1; rc=$?
echo "suite rc=$rc"; tail -2 $O/gpu_suite.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench.json'))
print('value', d['value'], 'ms/step', d['ms_per_step'], 'frac', d['roofline']['frac'], 'kinds', d['kinds_ms'])
print('c4', d['c4_secondary']['value'], 'cpu', d['cpu_baseline']['value'])
"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --fp16-steps 0 --c4-secondary 0 > $O/bench_under_rocprof.json 2> $O/kt.err || { tail -20 $O/kt.err; exit 1; }
cp "$(find $O/kt -name '*kernel_stats.csv' | head -1)" $O/kernel_stats.csv
head -8 $O/kernel_stats.csv | cut -c1-160
rm -rf $O/kt
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C -d $O/pmc_$C -o run --output-format csv -- python bench.py --utts 20 --steps 1 --warmup 0 --cpu-seconds 0 --no-profile --fp16-steps 0 --finetune-steps 0 --c4-secondary 0 > /dev/null 2> $O/pmc_$C.err || { tail -5 $O/pmc_$C.err; exit 1; }
done
python tools/pmc_summary.py "$(dirname "$(find $O/pmc_FETCH_SIZE -name '*counter_collection.csv' | head -1)")" "$(dirname "$(find $O/pmc_WRITE_SIZE -name '*counter_collection.csv' | head -1)")" $O/pmc_gemm_traffic_fp16x3.json > /dev/null
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_mfma -o run --output-format csv -- python bench.py --utts 20 --steps 1 --warmup 0 --cpu-seconds 0 --no-profile --fp16-steps 0 --finetune-steps 0 --c4-secondary 0 > /dev/null 2> $O/pmc_mfma.err || { tail -5 $O/pmc_mfma.err; exit 1; }
python tools/pmc_mfma.py "$(dirname "$(find $O/pmc_mfma -name '*counter_collection.csv' | head -1)")" $O/pmc_mfma.json > /dev/null
python -c "
import json
t=json.load(open('$O/pmc_gemm_traffic_fp16x3.json')); m=json.load(open('$O/pmc_mfma.json'))
for k in ('qkv','oproj','ffn1','ffn2'):
    e=t.get(k,{}); print(k, 'fetch/row', round((e.get('fetch_size_bytes_per_row') or 0)/1024,2), 'KB  write/row', round((e.get('write_size_bytes_per_row') or 0)/1024,2), 'KB')
for k,v in m.items():
    if k.startswith('x3s'): print(k, v)
"
rm -rf $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE $O/pmc_mfma
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; tail -1 $O/smoke.log
