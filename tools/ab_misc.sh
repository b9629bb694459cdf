# Interleaved end-to-end A/B of arbitrary settings in one GPU session (box-to-box spread ~5 %).
# usage: bash tools/ab_misc.sh ROUNDS "ENV=val[,ENV=val] [bench args]" ...   ('_' = no env)
set -eo pipefail
export TMPDIR=/tmp
R=$1; shift
mkdir -p gpurun_out/ab
for r in $(seq 1 "$R"); do
  i=0
  for setting in "$@"; do
    i=$((i+1))
    envs=$(echo "$setting" | cut -d' ' -f1 | tr ',' ' '); [ "$envs" = "_" ] && envs=""
    args=$(echo "$setting" | cut -s -d' ' -f2-)
    out=gpurun_out/ab/misc-$i-$r.json
    env $envs timeout -k 10 300 python bench.py --utts 100 --steps 3 --warmup 1 --cpu-seconds 0 $args > "$out" 2> "${out%.json}.err"
    echo "[$setting] round $r: $(python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(d['value'],d['kinds_ms'])" "$out")"
  done
done
