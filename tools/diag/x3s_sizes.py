"""Debug: x3s GEMM correctness across M (tiles per workgroup) and K."""
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
g = torch.Generator(device="cuda").manual_seed(1)
for M, N, K in ((512, 768, 768), (131072, 768, 768), (65536, 768, 768), (21760, 768, 768), (22016, 768, 768),
                (512, 768, 3072), (4096, 2304, 768)):
    A = torch.randn(M, K, device="cuda", generator=g)
    W = torch.randn(N, K, device="cuda", generator=g) * 0.05
    b = torch.randn(N, device="cuda", generator=g) * 0.1
    hi = A.half(); A2 = torch.cat([hi, ((A - hi.float()) * 64).half()], 1).contiguous()
    wh = W.half(); W2 = torch.cat([wh, ((W - wh.float()) * 64).half()], 1).contiguous()
    ref = A @ W.t() + b
    res = []
    for dbg in (0, 15, 9):
        out = torch.full((M, N), float("nan"), device="cuda")
        rc = fn(32, dbg, A2.data_ptr(), W2.data_ptr(), b.data_ptr(), out.data_ptr(), M, N, K, st)
        torch.cuda.synchronize()
        err = ((out - ref).abs().amax(1) / ref.abs().max())
        bad = (err > 1e-4).nonzero().flatten()
        res.append((dbg, rc, float(err.max()), int(bad.numel()), int(bad[0]) if bad.numel() else -1))
    print(M, N, K, "tiles", (M // 256) * (N // 256), res, flush=True)
