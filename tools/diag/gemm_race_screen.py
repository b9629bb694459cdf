"""Race screen for the persistent GEMM's wave schedule (younger half at s_setprio 1 and one
MFMA substep behind; wave-private epilogue slabs without the epilogue barrier): the production
variants must be BITWISE equal to the barrier-synchronised baseline (same MFMA order per
accumulator), over many random inputs, the four BERT projection shapes and row counts with
partial tile waves.  One process, no retries.
usage: python tools/diag/gemm_race_screen.py [reps]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import __graft_entry__  # noqa: E402

__graft_entry__._import_pkg()
from asr_rescoring_amd import _lib  # noqa: E402

# (production cfg, baseline cfg): 21 = bias, prio + stagger + private slab; 18 = GELU, prio +
# stagger; 9 / 11 = VAR 0 (barrier-synchronised, no priority)
PAIRS = {"bias": (21, 9), "gelu": (18, 11)}
SHAPES = [("qkv", 2304, 768, "bias"), ("oproj", 768, 768, "bias"), ("ffn1", 3072, 768, "gelu"),
          ("ffn2", 768, 3072, "bias")]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    lib = _lib.load()
    fn = lib.rs_debug_gemm
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_int] * 3 + [ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    st = torch.cuda.current_stream().cuda_stream
    bad = 0
    for M in (256 * 937, 65536, 262144):
        for name, N, K, kind in SHAPES:
            prod, base = PAIRS[kind]
            W = (torch.rand(N, K, device=dev, generator=g) * 2 - 1).half()
            b = torch.rand(N, device=dev, generator=g)
            o1 = torch.empty(M, N, device=dev, dtype=torch.float16)
            o2 = torch.empty_like(o1)
            diff = 0
            for r in range(reps):
                A = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).half()
                o1.fill_(float("nan"))
                o2.fill_(float("nan"))
                assert fn(prod, 0, A.data_ptr(), W.data_ptr(), b.data_ptr(), o1.data_ptr(), M, N, K, st) == 0
                assert fn(base, 0, A.data_ptr(), W.data_ptr(), b.data_ptr(), o2.data_ptr(), M, N, K, st) == 0
                torch.cuda.synchronize()
                if not torch.equal(o1.view(torch.int16), o2.view(torch.int16)):
                    diff += 1
            bad += diff
            print(f"M={M:7d} {name:5s} N={N} K={K}: {reps - diff}/{reps} bitwise equal", flush=True)
    print("RACE SCREEN", "PASS" if bad == 0 else f"FAIL ({bad} mismatching runs)")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
