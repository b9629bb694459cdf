# trainer GEMM 64x64 configs: parity, timing against cfg 0 / 5 / torch, split sweep
set -o pipefail
O=gpurun_out/r3r; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_sgemm.py -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
SG_CFGS=0,5,7,8 timeout -k 10 300 python -u tools/sgemm_bench.py > $O/sgemm.jsonl 2>&1 || exit 1
tail -1 $O/sgemm.jsonl
for s in 1 2 4 8; do
  SG_CFGS=7,8 RS_SGEMM_SPLITS=$s timeout -k 10 200 python -u tools/sgemm_bench.py > $O/split$s.jsonl 2>&1 || exit 1
  tail -1 $O/split$s.jsonl
done
