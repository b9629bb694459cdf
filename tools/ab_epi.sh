set -e
mkdir -p gpurun_out/ab
timeout -k 10 400 python -m pytest tests/test_gpu_bert.py -x -q 2>&1 | tail -2
for r in 1 2; do for m in none f16 all; do
  RS_GEMM_NT=$m timeout -k 10 200 python bench.py --utts 20 --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/ab/$m$r.json 2>/dev/null
done; done
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/ab/*.json")):
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d["value"], d.get("kinds_ms"))
PY
