"""Is the split-operand GEMM's result for a row independent of the row's position (tile /
lane)?  C(roll(A, s)) vs roll(C(A), s), bitwise, for the 16x16 (dbg 0) and 32x32 (dbg 19)
forms (diagnostic)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import __graft_entry__  # noqa: E402

__graft_entry__._import_pkg()
from asr_rescoring_amd import _lib  # noqa: E402

lib = _lib.load()
fn = lib.rs_debug_gemm
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_int] * 3 + [ctypes.c_void_p]
st = torch.cuda.current_stream().cuda_stream
g = torch.Generator(device="cuda").manual_seed(0)
M, N, K = 4096, 768, 256


def split2(x):
    hi = x.half()
    return torch.cat([hi, ((x - hi.float()) * 64.0).half()], dim=1).contiguous()


A = torch.randn(M, K, device="cuda", generator=g)
W = torch.randn(N, K, device="cuda", generator=g) * 0.05
b = torch.randn(N, device="cuda", generator=g) * 0.1
W2 = split2(W)
for dbg in (0, 19, 16):
    for shift in (1, 16, 32, 64, 128, 256):
        outs = []
        for s in (0, shift):
            A2 = split2(torch.roll(A, s, 0))
            o = torch.empty(M, N, device="cuda")
            assert fn(32, dbg, A2.data_ptr(), W2.data_ptr(), b.data_ptr(), o.data_ptr(), M, N, K, st) == 0
            torch.cuda.synchronize()
            outs.append(torch.roll(o, -s, 0))
        d = (outs[0] != outs[1]).any(dim=1)
        rows = torch.nonzero(d).flatten()
        print(f"dbg {dbg} shift {shift}: {int(d.sum())} of {M} rows differ; first {rows[:8].tolist()}; "
              f"max abs {float((outs[0] - outs[1]).abs().max()):.3e}", flush=True)
