#!/bin/bash
# Round 5: where the claimed-panel build loses 2 % — kernel trace + stamps, committed build vs new.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5m; rm -rf $O; mkdir -p $O
for v in head new; do
  if [ $v = head ]; then L=ab/librescore_head.so; else L=asr-rescoring_amd/librescore.so; fi
  RS_LIBRESCORE=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python -u tools/env_ab.py 100 2 '' > $O/prof_$v.txt 2>&1 || exit 1
  RS_LIBRESCORE=$L timeout -k 10 200 python -u tools/stamps.py 100 > $O/stamps_$v.txt 2>&1 || exit 1
done
python - <<'PY'
import csv, glob
for v in ("head", "new"):
    f = glob.glob(f"gpurun_out/r5m/prof_{v}/**/*kernel_stats.csv", recursive=True)
    rows = list(csv.DictReader(open(f[0])))
    for r in rows:
        n = r["Name"]
        if "gemm_x3s" in n or "attn" in n:
            print(v, n[:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us avg", round(float(r["TotalDurationNs"]) / 1e6, 1), "ms")
PY
for v in head new; do echo "== stamps $v"; grep -v amdgpu.ids gpurun_out/r5m/stamps_$v.txt | tail -12; done
