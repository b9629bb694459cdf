export TMPDIR=/tmp
mkdir -p gpurun_out/dd
timeout -k 10 600 python -u -m pytest tests/test_gpu_bert.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/dd/t.log 2>&1 || { tail -30 gpurun_out/dd/t.log; exit 1; }
tail -2 gpurun_out/dd/t.log
bash tools/ab_env.sh RS_DEDUP "0 1" 2 100
