"""Summarise rocprofv3 PMC runs of the GEMM kernels into per-row HBM traffic.

usage: python tools/pmc_summary.py <fetch_dir> <write_dir> <out.json>

FETCH_SIZE / WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE reports half the bytes of a wide
coalesced read stream (MI355X_MICROARCH.md §HBM), so fetch bytes = 2 x 1024 x FETCH_SIZE;
WRITE_SIZE is exact for 16-byte-per-lane stores.  Rows per launch: from the grid for
gemm_f16_kernel (blocks = (M_pad / BM) x (N / BN)); the persistent kernel's grid is the CU
count, so its rows come from its exact fp16 output bytes (N x 2 per row, same dispatch
order in both passes of the same command).  Infinity-Cache hits are counted too (the
counters sit on the L2's fabric side), so these are "beyond-L2" bytes, an upper bound on
HBM bytes.
"""
import collections
import csv
import json
import os
import re
import sys

EPI_N = {0: ("qkv", 2304), 1: ("ffn1", 3072), 3: ("res_f32", 768), 6: ("ffn2", 768),
         2: ("head_transform", 768), 4: ("decoder", 21248)}
OPROJ_TAG = 65536          # VAR bit of the O-projection instance of the persistent kernel
FFN2_TAG = 131072          # VAR bit of the BertOutput instance (fp16-output FFN2, RS_LNRES_DEFER=2)
RE_GEMM = re.compile(r"gemm_f16_kernelILi(\d+)ELi(\d+)ELi\d+ELi\d+ELi\d+ELi\d+ELi(\d+)E")
RE_PERSIST = re.compile(r"gemm_persist_kernelILi(\d+)ELi(\d+)E")
RE_X3S = re.compile(r"gemm_x3s_kernelILi(\d+)ELi(\d+)E")
# split-operand fp16x3 GEMMs: QKV, O-projection and FFN2 are one template instance (fp32
# output, EPI 5), told apart by dispatch order around the FFN1 instance (EPI 1): the fp32
# dispatch just before an FFN1 is the O-projection, the one just after it FFN2, the rest QKV
# (incl. the last layer's K/V and Q launches); rows from the output bytes (fp32: 4 N per row,
# FFN1: the two-part GELU image, 2 x 2 F per row)
X3S_OUT_BYTES = {"qkv": 4 * 2304, "oproj": 4 * 768, "ffn2": 4 * 768, "ffn1": 4 * 3072}


def label_x3s(epis):
    lab = []
    for i, e in enumerate(epis):
        if e == 1:
            lab.append("ffn1")
        elif i + 1 < len(epis) and epis[i + 1] == 1:
            lab.append("oproj")
        elif i > 0 and epis[i - 1] == 1:
            lab.append("ffn2")
        else:
            lab.append("qkv")
    return lab


def load(d):
    f = [os.path.join(d, x) for x in os.listdir(d) if x.endswith("counter_collection.csv")][0]
    return list(csv.DictReader(open(f)))


def main():
    fetch_dir, write_dir, out = sys.argv[1:4]
    # per (name, counter): list of (bytes, rows or None) in dispatch order
    res = collections.defaultdict(lambda: collections.defaultdict(list))
    x3s = {}
    for d, cname in ((fetch_dir, "FETCH_SIZE"), (write_dir, "WRITE_SIZE")):
        rows_x = []
        for r in load(d):
            if r["Counter_Name"] != cname:
                continue
            byt = float(r["Counter_Value"]) * 1024 * (2 if cname == "FETCH_SIZE" else 1)
            mx = RE_X3S.search(r["Kernel_Name"])
            if mx:
                rows_x.append((int(r.get("Dispatch_Id", len(rows_x))), int(mx.group(1)), byt))
                continue
            m, mp = RE_GEMM.search(r["Kernel_Name"]), RE_PERSIST.search(r["Kernel_Name"])
            if m:
                bm, bn, epi = int(m.group(1)), int(m.group(2)), int(m.group(3))
                name, n = EPI_N.get(epi, (f"epi{epi}", None))
                blocks = int(r["Grid_Size"]) // int(r["Workgroup_Size"])
                rows = blocks // (n // bn) * bm if n else None
            elif mp:
                tagv = int(mp.group(2))
                name, n = ("oproj", 768) if tagv & OPROJ_TAG else ("ffn2", 768) if tagv & FFN2_TAG else \
                    EPI_N.get(int(mp.group(1)), (f"epi{mp.group(1)}", None))
                rows = None                      # filled from the WRITE pass below
            else:
                continue
            res["persist:" + name if mp else name][cname].append((byt, rows))
        rows_x.sort()
        x3s[cname] = list(zip(label_x3s([e for _, e, _ in rows_x]), [b for _, _, b in rows_x]))
    if x3s.get("WRITE_SIZE"):
        wr = x3s["WRITE_SIZE"]
        for cname, seq in x3s.items():
            for i, (name, byt) in enumerate(seq):
                rows = wr[i][1] / X3S_OUT_BYTES[name] if i < len(wr) and wr[i][0] == name else None
                res["x3s:" + name][cname].append((byt, rows))
    for name, d in res.items():
        if name.startswith("persist:") and "WRITE_SIZE" in d:
            n = dict(list(EPI_N.values()) + [("oproj", 768)])[name.split(":", 1)[1]]
            rows = [b / (2 * n) for b, _ in d["WRITE_SIZE"]]
            for cname in d:
                d[cname] = [(b, rows[i] if i < len(rows) else None) for i, (b, _) in enumerate(d[cname])]
    summary = {}
    for name, d in res.items():
        e = {}
        for cname, vals in d.items():
            tot_b = sum(v[0] for v in vals)
            tot_r = sum(v[1] for v in vals if v[1])
            e[cname.lower() + "_bytes_per_launch"] = tot_b / len(vals)
            e[cname.lower() + "_bytes_per_row"] = tot_b / tot_r if tot_r else None
            e["launches"] = len(vals)
        summary[name.replace("persist:", "").replace("x3s:", "")] = e
    summary["_note"] = ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), gfx950 FETCH_SIZE x2 "
                        "correction; rows per launch from the grid size (persistent and split-operand "
                        "kernels: from their output bytes, so padded rows count as rows)")
    json.dump(summary, open(out, "w"), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
