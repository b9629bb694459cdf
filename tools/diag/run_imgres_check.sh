export TMPDIR=/tmp
mkdir -p gpurun_out/img
timeout -k 10 600 python -u -m pytest tests/test_gpu_bert.py tests/test_gpu_bertscore.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/img/t.log 2>&1 || { tail -30 gpurun_out/img/t.log; exit 1; }
tail -2 gpurun_out/img/t.log
SHAPES=3072x768 VARIANTS=x3s16-gelu2,x3s16-gelu2-late timeout -k 10 200 python -u tools/x3s_bench.py > gpurun_out/img/b.txt 2>&1 && cat gpurun_out/img/b.txt
bash tools/ab_env.sh RS_X3S_IMGRES "0 1" 2 100
