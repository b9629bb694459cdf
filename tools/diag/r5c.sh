#!/bin/bash
# round 5 GPU session c: LayerNorm-GEMM spill fix (new build) vs the round-4 build, interleaved;
# stamp shares; GPU parity tests of the touched paths
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5c; rm -rf $O; mkdir -p $O
for r in 1 2 3; do
  for L in r4 new; do
    if [ $L = r4 ]; then export RS_LIBRESCORE=$PWD/ab/librescore_r4.so; else unset RS_LIBRESCORE; fi
    timeout -k 10 300 python -u bench.py --utts 100 --steps 2 --warmup 1 --cpu-seconds 0 --fp16-steps 0 --finetune-steps 0 --c4-secondary 0 > $O/b_${L}_$r.json 2> $O/b_err.log || { tail -20 $O/b_err.log; exit 1; }
    echo "$L round $r: $(python -c "import json;d=json.load(open('$O/b_${L}_$r.json'));print(d['value'], d['kinds_ms'])")"
  done
done
unset RS_LIBRESCORE
timeout -k 10 300 python -u tools/env_ab.py 100 3 '' 'RS_LNGANG=xcd' > $O/env_ab.txt 2>&1 || { tail -20 $O/env_ab.txt; exit 1; }
tail -2 $O/env_ab.txt
timeout -k 10 300 python -u tools/stamps.py 50 > $O/stamps.txt 2>&1 || { tail -20 $O/stamps.txt; exit 1; }
timeout -k 10 300 python -u tools/stamps.py 50 xcd > $O/stamps_xcd.txt 2>&1 || { tail -20 $O/stamps_xcd.txt; exit 1; }
cat $O/stamps.txt $O/stamps_xcd.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_bert.py tests/test_gpu_robust.py tests/test_gpu_gemm.py tests/test_gpu_configs.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -3 $O/pytest.log
