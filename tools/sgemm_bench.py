"""Trainer fp32 GEMM (k_sgemm.hip, rs_debug_sgemm) vs torch fp32 matmul (rocBLAS / hipBLASLt)
at the bert-base training shapes: forward / dgrad / wgrad of each Linear and the tied MLM
decoder, for a 1.1k-token MLM batch and a 5.3k-token RescoreBert batch.
Usage: python tools/sgemm_bench.py"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__  # noqa: E402

__graft_entry__._import_pkg()
from asr_rescoring_amd import _lib  # noqa: E402


def main():
    lib = _lib.load()
    fn = lib.rs_debug_sgemm
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int] * 3 + [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                        ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    st = torch.cuda.current_stream().cuda_stream

    def timed(f, reps=20):
        for _ in range(3):
            f()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            f()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps
    tot_mine = tot_ref = 0.0
    for T in (1100, 5300):
        for (O, I) in [(2304, 768), (768, 768), (3072, 768), (768, 3072), (21128, 768)]:
            if O == 21128 and T > 2000:
                continue
            X = torch.randn(T, I, device="cuda")
            W = torch.randn(O, I, device="cuda") * 0.05
            dY = torch.randn(T, O, device="cuda") * 1e-3
            Y = torch.empty(T, O, device="cuda")
            dX = torch.empty(T, I, device="cuda")
            dW = torch.empty(O, I, device="cuda")
            for form, mine, ref in [
                ("fwd", lambda: fn(T, O, I, X.data_ptr(), I, 1, W.data_ptr(), I, 1, Y.data_ptr(), O, 0, st),
                 lambda: torch.matmul(X, W.t(), out=Y)),
                ("dgrad", lambda: fn(T, I, O, dY.data_ptr(), O, 1, W.data_ptr(), I, 0, dX.data_ptr(), I, 0, st),
                 lambda: torch.matmul(dY, W, out=dX)),
                ("wgrad", lambda: fn(O, I, T, dY.data_ptr(), O, 0, X.data_ptr(), I, 0, dW.data_ptr(), I, 0, st),
                 lambda: torch.matmul(dY.t(), X, out=dW))]:
                a, b = timed(mine), timed(ref)
                fl = 2.0 * T * O * I
                tot_mine += a
                tot_ref += b
                print(json.dumps({"tokens": T, "out": O, "in": I, "form": form, "ms_native": round(a, 4),
                                  "ms_torch": round(b, 4), "tflops_native": round(fl / a / 1e9, 1),
                                  "tflops_torch": round(fl / b / 1e9, 1)}), flush=True)
    print(json.dumps({"total_ms_native": round(tot_mine, 3), "total_ms_torch": round(tot_ref, 3)}))


if __name__ == "__main__":
    main()
