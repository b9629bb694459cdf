"""Where the split-operand GEMM's epilogue time goes (round 4 probe, timing only).

Variants of gemm_x3s_kernel through rs_debug_gemm (cfg 32 fp32 out, cfg 31 GELU image):
  prod     the production kernel
  nowait   the K loop never waits for its DMA, so the next tile never waits for this tile's stores
  alias    every tile stores onto row panel 0 (no HBM write burst; L2-resident lines)
  nw+al    both
  noepi    no stores (bias / GELU math kept)
(The round-5 PROBE=scale variants — no in-register operand scaling — were removed with their
kernel bits; the numbers stay in profiles/r5t_x3s_scale.txt.)  Needs the RS_DIAG build
(python asr-rescoring_amd/build.py --diag); operands are random interleaved images.
Rounds interleaved in one process; medians.  TF/s of MFMA work (3 x 2MNK).
Usage: python tools/x3s_epi_probe.py [M] [rounds]
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# the timing-diagnostic build (build.py --diag): the wrong-results GEMM variants / the stamp build
os.environ.setdefault("RS_LIBRESCORE", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                    "asr-rescoring_amd", "librescore_diag.so"))
import __graft_entry__  # noqa: E402

__graft_entry__._import_pkg()
from asr_rescoring_amd import _lib  # noqa: E402


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    lib = _lib.load()
    fn = lib.rs_debug_gemm
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_int] * 3 + [ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    st = torch.cuda.current_stream().cuda_stream
    shapes = ((2304, 768), (3072, 768), (768, 3072))
    if os.environ.get("SHAPES"):
        shapes = [tuple(int(v) for v in x.split("x")) for x in os.environ["SHAPES"].split(",")]
    for N, K in shapes:
        A2 = torch.randn(M, 2 * K, device=dev, generator=g).half()
        W2 = (torch.randn(N, 2 * K, device=dev, generator=g) * 0.05).half()
        b = torch.randn(N, device=dev, generator=g) * 0.1
        out32 = torch.empty(M, N, device=dev)
        img = torch.empty(M, 2 * N, device=dev, dtype=torch.float16)
        fl = 3 * 2.0 * M * N * K
        var = {"f32": (32, out32, {"prod": 0, "nowait": 50, "alias": 51, "nw+al": 53, "noepi": 20}),
               "gelu2": (31, img, {"prod": 0, "nowait": 50, "alias": 51, "nw+al": 53, "noepi": 52})}
        if os.environ.get("PROBE") == "bare":
            var = {"f32": (32, out32, {"prod": 0, "noepi": 20, "bare": 3})}
        times = {}
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(rounds):
            for kind, (cfg, o, dd) in var.items():
                for name, d in dd.items():
                    call = lambda: fn(cfg, d, A2.data_ptr(), W2.data_ptr(), b.data_ptr(), o.data_ptr(), M, N, K, st)  # noqa
                    for _ in range(2):
                        assert call() == 0
                    e0.record()
                    for _ in range(8):
                        assert call() == 0
                    e1.record()
                    torch.cuda.synchronize()
                    times.setdefault(f"{kind}-{name}", []).append(e0.elapsed_time(e1) / 8)
        res = {k: fl / (sorted(v)[len(v) // 2] * 1e-3) / 1e12 for k, v in times.items()}
        ms = {k: sorted(v)[len(v) // 2] for k, v in times.items()}
        print(f"M={M} N={N} K={K}: " + "  ".join(f"{k} {v:7.1f}TF {ms[k]:.3f}ms" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
