"""GEMM microbenchmark of librescore's fp16 MFMA kernel at the BERT projection shapes.

Runs every tile configuration with the diagnostic DBG bits (0 full, 1 no K-loop staging,
2 no epilogue, 3 neither) via ``rs_debug_gemm`` and prints TFLOP/s (HIP events on the
current stream, random [-1, 1) operands).  Usage: python tools/gemm_bench.py [M]
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__  # noqa: E402

__graft_entry__._import_pkg()
from asr_rescoring_amd import _lib  # noqa: E402


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
    cfgs = [int(c) for c in os.environ.get("CFGS", "0,1,2,3").split(",")]
    lib = _lib.load()
    fn = lib.rs_debug_gemm
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_int] * 3 + [ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    shapes = [(2304, 768), (768, 768), (3072, 768), (768, 3072)]
    if os.environ.get("SHAPES"):
        shapes = [tuple(int(v) for v in x.split("x")) for x in os.environ["SHAPES"].split(",")]
    dbgs = tuple(int(d) for d in os.environ.get("DBGS", "0,1,2,3").split(","))
    for N, K in shapes:
        A = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).half()
        W = (torch.rand(N, K, device=dev, generator=g) * 2 - 1).half()
        b = torch.rand(N, device=dev, generator=g)
        out = torch.empty(M, N, device=dev, dtype=torch.float16)
        ref = None
        rounds = int(os.environ.get("ROUNDS", "1"))
        for cfg in cfgs:
            # dbg variants interleaved, ROUNDS times; median per variant (box clocks drift)
            allres = [[_time(fn, cfg, dbg, A, W, b, out, M, N, K) for dbg in dbgs] for _ in range(rounds)]
            res = [sorted(col)[len(col) // 2] for col in zip(*allres)]
            if ref is None:
                ref = (A[:4096].float() @ W.float().t() + b).half()
            for dbg in dbgs:
                if cfg in (11, 12, 14, 16, 18, 20, 22, 24):      # GELU epilogue: compare against gelu(ref)
                    _time(fn, cfg, dbg, A, W, b, out, M, N, K, reps=1)
                    gl = torch.nn.functional.gelu(ref.float()).half()
                    assert (out[:4096].float() - gl.float()).abs().max().item() < 0.05 * K ** 0.5
                elif dbg in CHECKED:
                    _time(fn, cfg, dbg, A, W, b, out, M, N, K, reps=1)
                    err = (out[:4096].float() - ref.float()).abs().max().item()
                    assert err < 0.05 * K ** 0.5, (cfg, dbg, err)
            print(f"M={M} N={N} K={K} cfg={cfg}: " + "  ".join(f"{NAMES.get(d, d)} {v:7.1f}" for d, v in zip(dbgs, res))
                  + " TF/s", flush=True)


NAMES = {0: "full", 1: "nostage", 2: "noepi", 3: "neither", 4: "ilv", 6: "ilv-noepi", 8: "l2store", 16: "nostore",
         32: "direct", 40: "direct-l2", 64: "nt", 96: "direct-nt", 128: "pipe", 131: "pipe-neither", 192: "pipe-nt", 256: "fl", 320: "fl-nt", 259: "fl-neither", 704: "pipe-nt-nowait", 194: "pipe-noepi", 706: "pipe-noepi-nowait", 1216: "xk-nt", 1218: "xk-noepi", 1219: "xk-neither", 2240: "pp-nt", 6336: "pp-prio-nt", 2242: "pp-noepi", 2243: "pp-neither", 208: "pipe-nostore", 200: "pipe-nt-l2", 160: "pipe-direct", 8320: "m16-pipe", 8384: "m16-pipe-nt", 8323: "m16-neither", 8322: "m16-noepi", 8321: "m16-nostage", 270464: "m16-pipe-prio"}
CHECKED = (0, 4, 32, 64, 96, 128, 192, 256, 320, 1216, 2240, 6336, 160, 8320, 8384, 270464)      # variants that store the real result


def _time(fn, cfg, dbg, A, W, b, out, M, N, K, reps=10):
    st = torch.cuda.current_stream().cuda_stream
    call = lambda: fn(cfg, dbg, A.data_ptr(), W.data_ptr(), b.data_ptr(), out.data_ptr(), M, N, K, st)  # noqa
    for _ in range(3 if reps > 1 else 0):
        assert call() == 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        assert call() == 0
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return 2.0 * M * N * K / (ms * 1e-3) / 1e12

if __name__ == "__main__":
    main()
