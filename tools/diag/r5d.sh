#!/bin/bash
# round 5 GPU session d: robustness tests (co-residency limit), the spill-free LayerNorm build vs
# round 4 (interleaved), RS_LNGANG A/B, PMC traffic + MFMA busy for ticket and xcd gangs
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5d; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_robust.py -m gpu -v -s --timeout 120 --timeout-method thread > $O/robust.log 2>&1
echo "robust rc=$?"; grep -E "PASS|FAIL|RS_EHIP after|passed|failed" $O/robust.log | tail -20
for r in 1 2; do
  for L in r4 new; do
    if [ $L = r4 ]; then export RS_LIBRESCORE=$PWD/ab/librescore_r4.so; else unset RS_LIBRESCORE; fi
    timeout -k 10 300 python -u bench.py --utts 100 --steps 2 --warmup 1 --cpu-seconds 0 --fp16-steps 0 --finetune-steps 0 --c4-secondary 0 > $O/b_${L}_$r.json 2> $O/b_err.log || { tail -20 $O/b_err.log; exit 1; }
    echo "$L round $r: $(python -c "import json;d=json.load(open('$O/b_${L}_$r.json'));print(d['value'], d['kinds_ms'])")"
  done
done
unset RS_LIBRESCORE
timeout -k 10 300 python -u tools/env_ab.py 100 4 '' 'RS_LNGANG=xcd' > $O/env_ab.txt 2>&1 || { tail -20 $O/env_ab.txt; exit 1; }
tail -2 $O/env_ab.txt
timeout -k 10 300 python -u tools/stamps.py 50 > $O/stamps.txt 2>&1 || { tail -20 $O/stamps.txt; exit 1; }
grep -v amdgpu.ids $O/stamps.txt
for G in ticket xcd; do
  for C in FETCH_SIZE WRITE_SIZE; do
    RS_LNGANG=$G timeout -k 10 300 rocprofv3 --pmc $C -d $O/pmc_${G}_$C -o run --output-format csv -- python bench.py --utts 20 --steps 1 --warmup 0 --cpu-seconds 0 --no-profile --fp16-steps 0 --finetune-steps 0 --c4-secondary 0 > /dev/null 2> $O/pmc_${G}_$C.err || { tail -5 $O/pmc_${G}_$C.err; exit 1; }
  done
  python tools/pmc_summary.py "$(dirname "$(find $O/pmc_${G}_FETCH_SIZE -name '*counter_collection.csv' | head -1)")" "$(dirname "$(find $O/pmc_${G}_WRITE_SIZE -name '*counter_collection.csv' | head -1)")" $O/pmc_traffic_$G.json > /dev/null
  RS_LNGANG=$G timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_${G}_mfma -o run --output-format csv -- python bench.py --utts 20 --steps 1 --warmup 0 --cpu-seconds 0 --no-profile --fp16-steps 0 --finetune-steps 0 --c4-secondary 0 > /dev/null 2> $O/pmc_${G}_mfma.err || { tail -5 $O/pmc_${G}_mfma.err; exit 1; }
  python tools/pmc_mfma.py "$(dirname "$(find $O/pmc_${G}_mfma -name '*counter_collection.csv' | head -1)")" $O/pmc_mfma_$G.json > /dev/null
  echo "== $G"; python -c "
import json
t=json.load(open('$O/pmc_traffic_$G.json')); m=json.load(open('$O/pmc_mfma_$G.json'))
for k in ('qkv','oproj','ffn1','ffn2'):
    e=t.get(k,{}); print(k, 'fetch/row', round((e.get('fetch_size_bytes_per_row') or 0)/1024,2), 'KB  write/row', round((e.get('write_size_bytes_per_row') or 0)/1024,2), 'KB')
for k,v in m.items():
    if k.startswith('x3s'): print(k, v)
"
done
rm -rf $O/pmc_*_FETCH_SIZE $O/pmc_*_WRITE_SIZE $O/pmc_*_mfma
