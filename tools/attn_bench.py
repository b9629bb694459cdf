"""Attention microbenchmark: librescore's ragged attention kernels on synthetic sequences.

Lengths T ~ U{lo..hi} (default 26..44, the C3 masked-copy lengths), random fp16 Q/K/V.
Prints per kernel kind: time per launch, effective HBM bandwidth (Q,K,V read + ctx write),
and max |err| vs a torch fp32 reference on the first sequences.
usage: python tools/attn_bench.py [n_seq] [lo] [hi]   (env KINDS=0,6,10)
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__  # noqa: E402

__graft_entry__._import_pkg()
from asr_rescoring_amd import _lib  # noqa: E402

NAMES = {0: "tr", 3: "mem1", 4: "mem4", 6: "attn16", 9: "x3-valu", 10: "x3v2-48", 11: "x3v2-64"}


def main():
    n_seq = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
    lo = int(sys.argv[2]) if len(sys.argv) > 2 else 26
    hi = int(sys.argv[3]) if len(sys.argv) > 3 else 44
    kinds = [int(k) for k in os.environ.get("KINDS", "0,6").split(",")]
    H, heads = 768, 12
    lib = _lib.load()
    fn = lib.rs_debug_attention
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 3 + [ctypes.c_int] * 3 + [ctypes.c_void_p] * 2
    rng = np.random.default_rng(0)
    T = rng.integers(lo, hi + 1, size=n_seq).astype(np.int32)
    row = np.concatenate([[0], np.cumsum(T)[:-1]]).astype(np.int32)
    rows = int(T.sum())
    dev = torch.device("cuda", 0)
    qkv = (torch.randn(rows, 3 * H, device=dev) * 0.5).half()
    ctx = torch.zeros(rows, H, device=dev, dtype=torch.float16)
    d_len = torch.from_numpy(T).to(dev)
    d_row = torch.from_numpy(row).to(dev)
    st = torch.cuda.current_stream().cuda_stream
    byts = rows * (3 * H + H) * 2
    # reference for the first few sequences
    refs = []
    for s in range(8):
        r0, t = int(row[s]), int(T[s])
        x = qkv[r0:r0 + t].float().view(t, 3, heads, 64)
        q, k, v = x[:, 0].transpose(0, 1), x[:, 1].transpose(0, 1), x[:, 2].transpose(0, 1)
        p = torch.softmax(q @ k.transpose(1, 2) * 0.125, dim=-1)
        refs.append((r0, t, (p @ v).transpose(0, 1).reshape(t, H)))
    # split-precision kinds (9, 10, 11): fp32 qkv [rows, 3H] in, three-part fp16 image [rows, 3H] out
    qkv32 = ctx3 = None
    if any(k in (9, 10, 11) for k in kinds):
        qkv32 = qkv.float()
        ctx3 = torch.zeros(rows, 3 * H, device=dev, dtype=torch.float16)
    for kind in kinds:
        x3 = kind in (9, 10, 11)
        qp, cp = (qkv32.data_ptr(), ctx3.data_ptr()) if x3 else (qkv.data_ptr(), ctx.data_ptr())
        call = lambda: fn(kind, qp, d_len.data_ptr(), d_row.data_ptr(), n_seq, H, heads, cp, st)  # noqa
        byts = rows * (3 * H * 4 + 3 * H * 2) if x3 else rows * (3 * H + H) * 2
        ctx.zero_()
        assert call() == 0
        torch.cuda.synchronize()
        if x3:
            ctx3.zero_()
            assert call() == 0
            torch.cuda.synchronize()
            # three-part image [hi | hi/64 | lo*64] (common.h put_split4, kx = 3): hi + lo / 64
            img = ctx3.float()
            out = img[:, :H] + img[:, 2 * H:3 * H] / 64.0
            err = max((out[r0:r0 + t] - ref).abs().max().item() for r0, t, ref in refs)
        else:
            err = max((ctx[r0:r0 + t].float() - ref).abs().max().item() for r0, t, ref in refs) if kind in (0, 6) else float('nan')
        for _ in range(3):
            call()
        res = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                call()
            e1.record()
            torch.cuda.synchronize()
            res.append(e0.elapsed_time(e1) / 10)
        ms = sorted(res)[2]
        print(f"attn {NAMES.get(kind, kind):5s} n_seq={n_seq} T={lo}..{hi}: {ms * 1e3:8.1f} us/launch "
              f"{byts / (ms * 1e-3) / 1e9:7.0f} GB/s  max|err|={err:.2e}", flush=True)


if __name__ == "__main__":
    main()
