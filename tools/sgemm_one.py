"""One trainer-GEMM shape, repeated, for rocprofv3 kernel traces / PMC passes: every tile
configuration listed in SG_CFGS (k_sgemm.hip kSgCfg) and torch's fp32 matmul of the same form,
REPS launches each.  Usage: python tools/sgemm_one.py M N K form   (form fwd | dgrad | wgrad,
M N K as the GEMM sees them: C[M][N] over K)"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__  # noqa: E402

__graft_entry__._import_pkg()
from asr_rescoring_amd import _lib  # noqa: E402


def main():
    M, N, K, form = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    reps = int(os.environ.get("REPS", "20"))
    lib = _lib.load()
    fn = lib.rs_debug_sgemm_cfg
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                        ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    st = torch.cuda.current_stream().cuda_stream
    C = torch.empty(M, N, device="cuda")
    if form == "fwd":       # A [M][K], B [N][K]
        A, B = torch.randn(M, K, device="cuda"), torch.randn(N, K, device="cuda") * 0.05
        mine = lambda c: fn(c, M, N, K, A.data_ptr(), K, 1, B.data_ptr(), K, 1, C.data_ptr(), N, 0, st)  # noqa
        ref = lambda: torch.matmul(A, B.t(), out=C)  # noqa
    elif form == "dgrad":   # A [M][K], B [K][N]
        A, B = torch.randn(M, K, device="cuda") * 1e-3, torch.randn(K, N, device="cuda") * 0.05
        mine = lambda c: fn(c, M, N, K, A.data_ptr(), K, 1, B.data_ptr(), N, 0, C.data_ptr(), N, 0, st)  # noqa
        ref = lambda: torch.matmul(A, B, out=C)  # noqa
    else:                   # A [K][M], B [K][N]
        A, B = torch.randn(K, M, device="cuda") * 1e-3, torch.randn(K, N, device="cuda")
        mine = lambda c: fn(c, M, N, K, A.data_ptr(), M, 0, B.data_ptr(), N, 0, C.data_ptr(), N, 0, st)  # noqa
        ref = lambda: torch.matmul(A.t(), B, out=C)  # noqa
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for c in [int(x) for x in os.environ.get("SG_CFGS", "0,12").split(",")] + ["torch"]:
        f = ref if c == "torch" else (lambda: mine(c))
        for _ in range(3):
            r = f()
            assert c == "torch" or r == 0
        torch.cuda.synchronize()
        e0.record()
        for _ in range(reps):
            f()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        print(f"{form} M={M} N={N} K={K} cfg={c}: {ms * 1e3:.1f} us  {2.0 * M * N * K / ms / 1e9:.1f} TF", flush=True)


if __name__ == "__main__":
    main()
