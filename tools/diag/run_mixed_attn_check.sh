export TMPDIR=/tmp
mkdir -p gpurun_out/mx
timeout -k 10 700 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_bert.py tests/test_gpu_bertscore.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/mx/t.log 2>&1 || { tail -30 gpurun_out/mx/t.log; exit 1; }
tail -2 gpurun_out/mx/t.log
for v in 0 1 0 1; do RS_ATTN_V2=$v timeout -k 10 300 python -u tools/bench_extra.py c4 2>/dev/null | tail -1 | cut -c1-300; done
