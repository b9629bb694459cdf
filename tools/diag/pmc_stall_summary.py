"""Stall breakdown per GEMM kernel from a rocprofv3 PMC database (tools/diag/pmc_stall.sh):
wave-cycle shares (parked on s_waitcnt / barrier, issue-stalled, issuing), LDS bank-conflict
share of LDS-array cycles, MFMA busy and clock.  usage: python pmc_stall_summary.py <db>..."""
import collections
import re
import sqlite3
import sys


def short(n):
    m = re.search(r"sgemm_f32_kernel<(true|false), (true|false), (\d+)>", n) or \
        re.search(r"sgemm_f32_kernelILb(\d)ELb(\d)ELi(\d+)E", n)
    if m:
        return f"sgemm_f32<{m.group(1)},{m.group(2)},mode{m.group(3)}>"
    m = re.search(r"sgemm_dma_kernelILb(\d)ELb(\d)ELi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)E", n)
    if m:
        return f"sgemm_dma<{m.group(1)},{m.group(2)},{m.group(3)}x{m.group(4)}x{m.group(6)},occ{m.group(7)}>"
    m = re.search(r"gemm_x3s_kernelILi(\d+)ELi(\d+)E", n)
    if m:
        return f"x3s<{m.group(1)},{m.group(2)}>"
    m = re.search(r"gemm_persist_kernelILi(\d+)ELi(\d+)E", n)
    if m:
        return f"persist<{m.group(1)},{m.group(2)}>"
    m = re.search(r"attn16x3v2_kernelILb(\d)ELi(\d+)E", n)
    if m:
        return f"attn16x3v2<dedup{m.group(1)},R{m.group(2)}>"
    m = re.search(r"gemm_f16_kernelILi(\d+)ELi(\d+)E.*?ELi(\d+)ELi(\d+)EEEv", n)
    if m:
        return f"plain<{m.group(1)}x{m.group(2)},epi{m.group(3)},var{m.group(4)}>"
    return n[:50]


for db in sys.argv[1:]:
    c = sqlite3.connect(db)
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = collections.defaultdict(float)
    seen = set()
    for name, cn, val, did, d in c.execute("select kernel_name, counter_name, value, dispatch_id, duration from counters_collection"):
        k = short(name)
        acc[k][cn] += val
        if (k, did) not in seen:
            seen.add((k, did))
            dur[k] += d
    for k, v in acc.items():
        wc = v["SQ_WAVE_CYCLES"] or 1
        gui = v["GRBM_GUI_ACTIVE"] / 8
        print(f"{k:38s} parked {v['SQ_WAIT_ANY'] / wc:5.1%}  issue-stall {v['SQ_WAIT_INST_ANY'] / wc:5.1%} "
              f"(lds {v['SQ_WAIT_INST_LDS'] / wc:5.1%})  issuing {v['SQ_ACTIVE_INST_ANY'] / wc:5.1%}  "
              f"lds-conflict {v['SQ_LDS_BANK_CONFLICT'] / max(v['SQ_LDS_IDX_ACTIVE'], 1):5.1%}  "
              f"mfma-busy {v['SQ_VALU_MFMA_BUSY_CYCLES'] / (4 * 256 * gui):5.1%}  clk {gui / dur[k]:.2f} GHz")
