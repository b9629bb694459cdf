"""Split-operand fp16x3 GEMM (gemm_x3s_kernel) vs the K-concatenated fp16x3 form.

Checks x3s against an fp32 matmul (rows sampled) and times, at the BERT projection shapes:
  x3s fp32 out (cfg 32), x3s GELU two-part image (cfg 31), x3s fp16 out (cfg 30),
  the persistent fp16 kernel over a K x 3 operand (cfg 9 / 11: the MFMA work of the
  K-concatenated fp16x3 form).
TF/s counted as MFMA work (3 x 2MNK for every variant).  Usage: python tools/x3s_bench.py [M]
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__  # noqa: E402

__graft_entry__._import_pkg()
from asr_rescoring_amd import _lib  # noqa: E402


def split2(x):
    hi = x.half()
    lo = ((x - hi.float()) * 64.0).half()
    return torch.cat([hi, lo], dim=1).contiguous()


def timed(fn, reps=10):
    for _ in range(3):
        assert fn() == 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        assert fn() == 0
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
    lib = _lib.load()
    fn = lib.rs_debug_gemm
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_int] * 3 + [ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    st = torch.cuda.current_stream().cuda_stream
    shapes = [(2304, 768), (768, 768), (3072, 768), (768, 3072)]
    if os.environ.get("SHAPES"):
        shapes = [tuple(int(v) for v in x.split("x")) for x in os.environ["SHAPES"].split(",")]
    for N, K in shapes:
        A = torch.randn(M, K, device=dev, generator=g)
        Wt = torch.randn(N, K, device=dev, generator=g) * 0.05
        b = torch.randn(N, device=dev, generator=g) * 0.1
        A2, W2 = split2(A), split2(Wt)
        ref = A[:2048] @ Wt.t() + b
        out32 = torch.empty(M, N, device=dev)
        out_img = torch.empty(M, 2 * N, device=dev, dtype=torch.float16)
        out16 = torch.empty(M, N, device=dev, dtype=torch.float16)
        call = lambda cfg, a, w, o, k, d=0: fn(cfg, d, a.data_ptr(), w.data_ptr(), b.data_ptr(), o.data_ptr(), M, N, k, st)  # noqa
        assert call(32, A2, W2, out32, K) == 0
        torch.cuda.synchronize()
        err32 = ((out32[:2048] - ref).abs().max() / ref.abs().max()).item()
        for d in (0, 5, 9, 10, 16, 17, 21, 26, 27, 28, 29):
            out32.zero_()
            assert call(32, A2, W2, out32, K, d) == 0
            torch.cuda.synchronize()
            err32 = max(err32, ((out32[:2048] - ref).abs().max() / ref.abs().max()).item())
        gl = torch.nn.functional.gelu(ref)
        errg = 0.0
        for d in (0, 16, 22, 27, 28, 29):
            out_img.zero_()
            assert call(31, A2, W2, out_img, K, d) == 0
            torch.cuda.synchronize()
            rec = out_img[:2048, :N].float() + out_img[:2048, N:].float() / 64.0
            errg = max(errg, ((rec - gl).abs().max() / gl.abs().max()).item())
        # whole-output checks of the 16x16 path against the production path (every row, so a
        # tile-order or last-tile defect shows): fp32, GELU image, fp16
        o2 = torch.empty_like(out32)
        assert call(32, A2, W2, out32, K, 19) == 0 and call(32, A2, W2, o2, K, 16) == 0
        torch.cuda.synchronize()
        err16 = ((o2 - out32).abs().max() / out32.abs().max()).item()
        i2 = torch.empty_like(out_img)
        assert call(31, A2, W2, out_img, K, 19) == 0 and call(31, A2, W2, i2, K, 16) == 0
        torch.cuda.synchronize()
        rec16 = lambda im: im[:, :N].float() + im[:, N:].float() / 64.0  # noqa: E731
        r0 = rec16(out_img)
        err16 = max(err16, ((rec16(i2) - r0).abs().max() / r0.abs().max()).item())
        h2 = torch.empty_like(out16)
        assert call(30, A2, W2, out16, K, 19) == 0 and call(30, A2, W2, h2, K, 16) == 0
        torch.cuda.synchronize()
        # fp16 outputs: the two accumulation orders (each ~1e-6 of max |C| from exact) may
        # round to neighbouring fp16 values: within one fp16 ulp of the value + 1e-5 max |C|
        d16 = (h2.float() - out16.float()).abs()
        bound = out16.float().abs() * 2 ** -10 + 1e-5 * out16.float().abs().max()
        assert bool((d16 <= bound).all()), (d16 / bound).max().item()
        # half-step stagger (dbg 40): bitwise equal to the production kernel on every output
        for cfg_s, o_a in ((32, out32), (31, out_img), (30, out16)):
            o_b = torch.empty_like(o_a)
            for dbg_s in ((40, 44) if cfg_s != 30 else (40,)):
                assert call(cfg_s, A2, W2, o_a, K, 0) == 0 and call(cfg_s, A2, W2, o_b, K, dbg_s) == 0
                torch.cuda.synchronize()
                assert torch.equal(o_a, o_b), f"stagger differs (cfg {cfg_s}, dbg {dbg_s})"
        # the K-concatenated form: K x 3 operand (values irrelevant to timing)
        A3 = torch.cat([A2, A2[:, :K]], dim=1).contiguous()
        W3 = torch.cat([W2, W2[:, :K]], dim=1).contiguous()
        fl = 3 * 2.0 * M * N * K
        res = {}
        variants = [("x3s-f32", 32, A2, W2, out32, K, 0), ("x3s-f32-nostage", 32, A2, W2, out32, K, 1),
                    ("x3s-f32-noepi", 32, A2, W2, out32, K, 2), ("x3s-f32-neither", 32, A2, W2, out32, K, 3),
                    ("x3s-f32-noprio", 32, A2, W2, out32, K, 4), ("x3s-f32-ilv", 32, A2, W2, out32, K, 5),
                    ("x3s-f32-ilv-noepi", 32, A2, W2, out32, K, 6), ("x3s-f32-ilv-noepi-nowait", 32, A2, W2, out32, K, 7),
                    ("x3s-f32-noepi-nowait", 32, A2, W2, out32, K, 8), ("x3s-f32-buf", 32, A2, W2, out32, K, 9),
                    ("x3s-f32-buf-ilv", 32, A2, W2, out32, K, 10), ("x3s-f32-prod", 32, A2, W2, out32, K, 0), ("x3s-f32-buf-ilv-noepi", 32, A2, W2, out32, K, 11),
                    ("x3s-f32-mf16diag", 32, A2, W2, out32, K, 12), ("x3s-f32-mf16diag-neither", 32, A2, W2, out32, K, 13),
                    ("x3s-f32-prod-neither", 32, A2, W2, out32, K, 14),
                    ("x3s16-f32", 32, A2, W2, out32, K, 16), ("x3s16-f32-noilv", 32, A2, W2, out32, K, 17),
                    ("x3s16-f32-neither", 32, A2, W2, out32, K, 18), ("x3s16-gelu2", 31, A2, W2, out_img, K, 16), ("x3s16-gelu2-late", 31, A2, W2, out_img, K, 22),
                    ("x3s16-f32-noepi", 32, A2, W2, out32, K, 20), ("x3s16-f32-noepi-Wonly", 32, A2, W2, out32, K, 23),
                    ("x3s16-f32-noepi-Aonly", 32, A2, W2, out32, K, 24),
                    ("x3s16-f32-noepi-dma4B", 32, A2, W2, out32, K, 25),
                    ("x3s16-f32-branchfree", 32, A2, W2, out32, K, 26), ("x3s16-gelu2-branchfree", 31, A2, W2, out_img, K, 26),
                    ("x3s-gelu2-prod", 31, A2, W2, out_img, K, 0),
                    ("x3s16-f32-spread", 32, A2, W2, out32, K, 27), ("x3s16-f32-noprio", 32, A2, W2, out32, K, 28),
                    ("x3s16-gelu2-spread", 31, A2, W2, out_img, K, 27),
                    ("x3s16-f32-olddma", 32, A2, W2, out32, K, 29), ("x3s16-gelu2-olddma", 31, A2, W2, out_img, K, 29), ("x3s16-gelu2-noprio", 31, A2, W2, out_img, K, 28), ("x3s16-f32-direct", 32, A2, W2, out32, K, 21),
                    ("x3s-gelu2", 31, A2, W2, out_img, K, 0), ("kcat-persist-f16", 9, A3, W3, out16, 3 * K, 0),
                    ("x3s16-f32-stag", 32, A2, W2, out32, K, 40), ("x3s16-f32-stag-neither", 32, A2, W2, out32, K, 41),
                    ("x3s16-f32-stag-noepi", 32, A2, W2, out32, K, 42), ("x3s16-f32-prodV-neither", 32, A2, W2, out32, K, 43),
                    ("x3s16-gelu2-stag", 31, A2, W2, out_img, K, 40), ("x3s16-f16-stag", 30, A2, W2, out16, K, 40),
                    ("x3s16-f16-prod", 30, A2, W2, out16, K, 0),
                    ("x3s16-f32-stagL", 32, A2, W2, out32, K, 44), ("x3s16-f32-stagL-noepi", 32, A2, W2, out32, K, 45),
                    ("x3s16-gelu2-stagL", 31, A2, W2, out_img, K, 44),
                    ("x3s16-f32-noepi-nowait", 32, A2, W2, out32, K, 46), ("x3s16-f32-stag-noepi-nowait", 32, A2, W2, out32, K, 47),
                    ("x3s16-f32-pfA", 32, A2, W2, out32, K, 48), ("x3s16-f32-pfA-noepi", 32, A2, W2, out32, K, 49),
                    ("x3s16-gelu2-pfA", 31, A2, W2, out_img, K, 48)]
        if os.environ.get("VARIANTS"):
            keep = os.environ["VARIANTS"].split(",")
            variants = [v for v in variants if v[0] in keep]
        for name, cfg, a, w, o, k, d in variants:
            ms = sorted(timed(lambda: call(cfg, a, w, o, k, d)) for _ in range(3))[1]
            res[name] = fl / (ms * 1e-3) / 1e12
        print(f"M={M} N={N} K={K}: err32 {err32:.2e} errgelu {errg:.2e} err16vs32 {err16:.2e}  " +
              "  ".join(f"{k} {v:7.1f}" for k, v in res.items()) + " TF/s (MFMA work)", flush=True)


if __name__ == "__main__":
    main()
