"""MFMA utilisation and effective clock per kernel from a rocprofv3 PMC pass with
SQ_VALU_MFMA_BUSY_CYCLES and GRBM_GUI_ACTIVE (MI355X_MICROARCH.md: the busy counter is in
cycles, 32 per v_mfma_f32_32x32x16; GRBM_GUI_ACTIVE is summed over the 8 XCDs).

  mfma_busy  = SQ_VALU_MFMA_BUSY_CYCLES / (4 SIMDs x n_CU x GRBM_GUI_ACTIVE / 8)
  clock_GHz  = GRBM_GUI_ACTIVE / 8 / kernel duration

usage: python tools/pmc_mfma.py <dir with *counter_collection.csv> <out.json> [n_cu=256]
"""
import collections
import csv
import json
import os
import re
import sys

EPI = {0: "qkv", 1: "ffn1", 2: "head_transform", 3: "res_f32(last layer)", 4: "decoder", 5: "qkv32", 6: "ffn2"}


def kname(n):
    m = re.search(r"gemm_x3s_kernelILi(\d+)ELi(\d+)E", n)
    if m:
        epi, var = int(m.group(1)), int(m.group(2))
        if epi == 7:
            return "x3s:ffn2+LN" if var & 67108864 else "x3s:oproj+LN"
        return "x3s:" + {5: "qkv(f32 out)", 1: "ffn1(GELU image)", 3: "f16 out"}.get(epi, str(epi))
    m = re.search(r"gemm_persist_kernelILi(\d+)ELi(\d+)E", n)
    if m and int(m.group(2)) & 65536:
        return "gemm_persist:oproj"
    if m and int(m.group(2)) & 131072:
        return "gemm_persist:ffn2"
    if m:
        return "gemm_persist:" + EPI.get(int(m.group(1)), m.group(1))
    m = re.search(r"gemm_f16_kernelILi\d+ELi\d+ELi\d+ELi\d+ELi\d+ELi\d+ELi(\d+)E", n)
    if m:
        return "gemm:" + EPI.get(int(m.group(1)), m.group(1))
    m = re.search(r"(attn_\w+?|ln_res_rows|ln_rows|embed_ln)_kernel", n)
    return m.group(1) if m else n[:40]


def main():
    d, out = sys.argv[1], sys.argv[2]
    n_cu = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    f = [os.path.join(d, x) for x in os.listdir(d) if x.endswith("counter_collection.csv")][0]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        k = kname(r["Kernel_Name"])
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
            acc[k]["ns"] += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
            acc[k]["n"] += 1
    res = {}
    for k, v in acc.items():
        g = v.get("GRBM_GUI_ACTIVE", 0.0)
        if g <= 0 or not v.get("ns"):
            continue
        res[k] = {"launches": int(v["n"]),
                  "mfma_busy": round(v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (4 * n_cu * g / 8), 4),
                  "clock_GHz": round(g / 8 / v["ns"], 3)}
    res["_note"] = "rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE; busy / (4 x n_CU x GRBM/8)"
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
