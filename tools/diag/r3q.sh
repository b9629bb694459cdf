# trainer end to end: native GEMMs vs the rocBLAS baseline, interleaved; a quick scoring sanity run
set -o pipefail
O=gpurun_out/r3q; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_bert.py -x -q --timeout 240 --timeout-method thread -k "golden or lnfuse" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  timeout -k 10 300 python -u tools/bench_extra.py c2train,mlmtrain > $O/native_r$r.jsonl 2>&1 || exit 1
  RS_TRAIN_ROCBLAS=1 timeout -k 10 300 python -u tools/bench_extra.py c2train,mlmtrain > $O/rocblas_r$r.jsonl 2>&1 || exit 1
done
for f in $O/native_r*.jsonl $O/rocblas_r*.jsonl; do grep -o '"workload": "[A-Za-z]*[^,]*\|"ms_per_step": [0-9.]*' $f | paste -sd' ' | sed "s#^#$(basename $f) #"; done
