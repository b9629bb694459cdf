"""Per-kernel summary of rocprofv3 CSV runs: kernel-trace stats (calls, average us) and, if given,
a FETCH_SIZE pass (beyond-L2 fetch per dispatch, gfx950 x2 correction), for the GEMM / attention
kernels.  usage: python tools/diag/kt_summary.py <trace_dir> [<fetch_dir>]"""
import collections
import csv
import glob
import sys


def short(n):
    for k, lab in (("gemm_x3s_kernelILi7ELi218103808", "x3s LN ffn2 xcd"), ("gemm_x3s_kernelILi7ELi150994944", "x3s LN oproj xcd"),
                   ("gemm_x3s_kernelILi7ELi83886080", "x3s LN ffn2 ticket"), ("gemm_x3s_kernelILi7ELi16777216E", "x3s LN oproj ticket"),
                   ("gemm_x3s_kernelILi1E", "x3s ffn1 gelu"), ("gemm_x3s_kernelILi5E", "x3s fp32 (qkv)"), ("attn", "attention"),
                   ("embed", "embed"), ("gemm_f16", "gemm_f16"), ("gemm_persist", "gemm_persist")):
        if k in n:
            return lab
    return None


tr = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)
agg = collections.defaultdict(lambda: [0, 0.0])
for r in csv.DictReader(open(tr[0])):
    s = short(r["Name"])
    if s:
        agg[s][0] += int(r["Calls"])
        agg[s][1] += float(r["TotalDurationNs"])
fetch = collections.defaultdict(lambda: [0, 0.0])
if len(sys.argv) > 2:
    f = glob.glob(sys.argv[2] + "/**/*counter_collection.csv", recursive=True)
    for r in csv.DictReader(open(f[0])):
        s = short(r["Kernel_Name"])
        if s and r["Counter_Name"] == "FETCH_SIZE":
            fetch[s][0] += 1
            fetch[s][1] += float(r["Counter_Value"]) * 2048
for s, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    fc, fb = fetch.get(s, (0, 0.0))
    print(f"{s:22s} calls {c:6d}  avg {t / c / 1e3:9.1f} us  total {t / 1e6:9.1f} ms"
          + (f"  fetch/dispatch {fb / fc / 1e6:8.1f} MB" if fc else ""))
