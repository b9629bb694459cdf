"""Per-kernel register / scratch / spill report of one .hip file (hipcc -Rpass-analysis):
python tools/kres.py asr-rescoring_amd/csrc/k_gemm.hip [name-substring]"""
import re
import subprocess
import sys

src = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
inc = __file__.rsplit("/tools/", 1)[0] + "/include"
r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-I", inc,
                    "-c", src, "-o", "/tmp/_kres.o", "-Rpass-analysis=kernel-resource-usage"],
                   capture_output=True, text=True)
cur = None
rows = []
for line in r.stderr.splitlines():
    m = re.search(r"remark: (?:\s*)(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|SGPRs Spill|VGPRs Spill|Occupancy \[waves/SIMD\]): (\S+)", line)
    if not m:
        if "error" in line:
            print(line)
        continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for d in rows:
    if pat in d["name"]:
        print(f'{d["name"][:90]:90s} vgpr {d.get("VGPRs")} agpr {d.get("AGPRs")} scratch {d.get("ScratchSize [bytes/lane]")} '
              f'vspill {d.get("VGPRs Spill")} sspill {d.get("SGPRs Spill")} occ {d.get("Occupancy [waves/SIMD]")}')
sys.exit(r.returncode)
