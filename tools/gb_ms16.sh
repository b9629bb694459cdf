set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/gb
CFGS=9,10,11,12 DBGS=0,1 ROUNDS=3 timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gb/persist.txt 2>&1
cat gpurun_out/gb/*.txt
