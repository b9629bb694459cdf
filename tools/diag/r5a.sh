#!/bin/bash
# round 5 GPU session a: parity of the K-loop residual LayerNorm GEMM (RS_LNKRES 1 default, 2, 0),
# in-process A/B of RS_LNKRES, and the new build against the round-4 build (ab/librescore_r4.so)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5a; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_bert.py tests/test_gpu_robust.py tests/test_gpu_gemm.py tests/test_gpu_configs.py -m gpu -q --deselect tests/test_gpu_robust.py::test_chunks_at_gang_rounds_match --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
RS_LNKRES=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_bert.py -m gpu -x -q -k "fp16x3 or lnfuse" --timeout 300 --timeout-method thread > $O/pytest_k2.log 2>&1 || { tail -30 $O/pytest_k2.log; exit 1; }
tail -2 $O/pytest_k2.log
timeout -k 10 300 python -u tools/env_ab.py 100 3 'RS_LNKRES=0' 'RS_LNKRES=1' 'RS_LNKRES=2' 'RS_LNKRES=1;RS_LNGANG=xcd' 'RS_LNKRES=0;RS_LNGANG=xcd' > $O/env_ab.txt 2>&1 || { tail -20 $O/env_ab.txt; exit 1; }
cat $O/env_ab.txt
for r in 1 2; do
  for L in r4 new; do
    if [ $L = r4 ]; then export RS_LIBRESCORE=$PWD/ab/librescore_r4.so; else unset RS_LIBRESCORE; fi
    timeout -k 10 300 python -u bench.py --utts 100 --steps 2 --warmup 1 --cpu-seconds 0 --fp16-steps 0 --finetune-steps 0 > $O/b_${L}_$r.json 2> $O/b_err.log || { tail -20 $O/b_err.log; exit 1; }
    echo "$L round $r: $(python -c "import json;d=json.load(open('$O/b_${L}_$r.json'));print(d['value'], d['kinds_ms'])")"
  done
done
unset RS_LIBRESCORE
