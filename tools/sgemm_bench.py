"""Trainer fp32 GEMM (k_sgemm.hip, rs_debug_sgemm_cfg) vs torch fp32 matmul (rocBLAS / hipBLASLt)
at the bert-base training shapes: forward / dgrad / wgrad of each Linear and the tied MLM
decoder, for a 1.1k-token MLM batch and a 5.3k-token RescoreBert batch; every tile
configuration named in SG_CFGS (default 0: 128x128, 11: 64x64 direct-to-register, 12: 128x128
software-pipelined)
and the shape's pick (-1), interleaved in
one process; SG_TOKENS picks the token counts (default 1100,5300).  Usage: python tools/sgemm_bench.py"""
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
    fn = lib.rs_debug_sgemm_cfg
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
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
    CFGS = (-1,) + tuple(int(c) for c in os.environ.get("SG_CFGS", "0,11,12").split(","))
    tot = {c: 0.0 for c in CFGS}
    tot_ref = 0.0
    for T in [int(x) for x in os.environ.get("SG_TOKENS", "1100,5300").split(",")]:
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
                ("fwd", lambda c: fn(c, T, O, I, X.data_ptr(), I, 1, W.data_ptr(), I, 1, Y.data_ptr(), O, 0, st),
                 lambda: torch.matmul(X, W.t(), out=Y)),
                ("dgrad", lambda c: fn(c, T, I, O, dY.data_ptr(), O, 1, W.data_ptr(), I, 0, dX.data_ptr(), I, 0, st),
                 lambda: torch.matmul(dY, W, out=dX)),
                ("wgrad", lambda c: fn(c, O, I, T, dY.data_ptr(), O, 0, X.data_ptr(), I, 0, dW.data_ptr(), I, 0, st),
                 lambda: torch.matmul(dY.t(), X, out=dW))]:
                fl = 2.0 * T * O * I
                ms = {c: [] for c in CFGS}
                mr = []
                for _ in range(3):                       # interleaved rounds, median
                    for c in CFGS:
                        ms[c].append(timed(lambda: mine(c)))
                    mr.append(timed(ref))
                med = {c: sorted(v)[1] for c, v in ms.items()}
                b = sorted(mr)[1]
                for c in CFGS:
                    tot[c] += med[c]
                tot_ref += b
                print(json.dumps({"tokens": T, "out": O, "in": I, "form": form, "ms_torch": round(b, 4),
                                  "ms_pick": round(med[-1], 4), "ms_cfg": [round(med[c], 4) for c in CFGS[1:]],
                                  "tflops_pick": round(fl / med[-1] / 1e9, 1),
                                  "tflops_torch": round(fl / b / 1e9, 1)}), flush=True)
    print(json.dumps({"total_ms_pick": round(tot[-1], 3), "total_ms_cfg": [round(tot[c], 3) for c in CFGS[1:]],
                      "total_ms_torch": round(tot_ref, 3), "pick_vs_torch": round(tot_ref / tot[-1], 3)}))


if __name__ == "__main__":
    main()
