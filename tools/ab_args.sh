# A/B of bench.py argument sets, interleaved in one GPU session (box-to-box spread ~5 %).
# usage: bash tools/ab_args.sh NAME "args A|args B|..." [rounds] [utts]
set -eo pipefail
export TMPDIR=/tmp
N=$1; IFS='|' read -ra SETS <<< "$2"; R=${3:-2}; U=${4:-100}
mkdir -p gpurun_out/ab
for r in $(seq 1 $R); do for i in "${!SETS[@]}"; do
  timeout -k 10 300 python bench.py --utts $U --steps 3 --warmup 1 --cpu-seconds 0 --fp16-steps 0 ${SETS[$i]} \
    > gpurun_out/ab/$N-$i-$r.json 2> gpurun_out/ab/$N-$i-$r.err
done; done
python - "$2" <<PY
import json, glob, sys
sets = sys.argv[1].split("|")
for f in sorted(glob.glob("gpurun_out/ab/$N-*.json")):
    i = int(f.rsplit("-", 2)[1])
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, repr(sets[i]), d["value"], d.get("kinds_ms"))
PY
