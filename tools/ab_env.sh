# A/B of an environment switch on the end-to-end bench, interleaved in one GPU session
# (box-to-box spread is ~5 %).  usage: bash tools/ab_env.sh VAR "valA valB" [rounds] [utts]
set -eo pipefail
export TMPDIR=/tmp
V=$1; VALS=$2; R=${3:-2}; U=${4:-100}
mkdir -p gpurun_out/ab
for r in $(seq 1 $R); do for v in $VALS; do
  env $V=$v timeout -k 10 300 python bench.py --utts $U --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/ab/$V-$v-$r.json 2> gpurun_out/ab/$V-$v-$r.err
done; done
python - <<PY
import json,glob
for f in sorted(glob.glob("gpurun_out/ab/$V-*.json")):
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d["value"], d.get("kinds_ms"))
PY
