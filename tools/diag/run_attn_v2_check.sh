export TMPDIR=/tmp
mkdir -p gpurun_out/av2
timeout -k 10 600 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_bert.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/av2/t.log 2>&1 || { tail -30 gpurun_out/av2/t.log; exit 1; }
tail -2 gpurun_out/av2/t.log
bash tools/ab_env.sh RS_ATTN_V2 "0 1" 2 100
