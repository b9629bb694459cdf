set -eo pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bert.py -x -q --timeout 300 --timeout-method thread 2>&1 | tail -2
RS_FFN2=f16 timeout -k 10 300 python -u -m pytest tests/test_gpu_bert.py -x -q --timeout 300 --timeout-method thread 2>&1 | tail -2
mkdir -p gpurun_out/ab
for r in 1 2; do
 for v in "RS_FFN2=resln" "RS_FFN2=f16" "RS_FFN2=f16 RS_GEMM_MS_PERSIST=0"; do
  n=$(echo $v | tr ' =' '__')
  env $v timeout -k 10 300 python bench.py --utts 100 --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/ab/$n-$r.json 2> gpurun_out/ab/$n-$r.err
 done
done
python - <<PY
import json,glob
for f in sorted(glob.glob("gpurun_out/ab/RS_FFN2*.json")):
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d["value"], d.get("kinds_ms"))
PY
