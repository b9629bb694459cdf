"""LayerNorm-family kernel microbenchmark (rs_debug_ln): GB/s of ln_rows, ln_res_rows (write
back / deferred), the two-block pass and its memory skeleton at the bench's chunk size.
Usage: python tools/ln_bench.py [rows]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__  # noqa: E402

__graft_entry__._import_pkg()
from asr_rescoring_amd import _lib  # noqa: E402

# bytes per row: reads + writes (H = 768)
BYTES = {0: 3072 + 1536 + 8, 1: 3072 + 1536 + 8 + 3072 + 1536 + 8, 2: 3072 + 1536 + 8 + 1536 + 8,
         3: 3072 + 2 * 1536 + 16 + 3072 + 1536 + 8, 4: 3072 + 2 * 1536 + 3072 + 1536}
NAMES = {0: "ln_rows", 1: "ln_res_rows", 2: "ln_res_rows(defer)", 3: "ln_res_rows(two-block)", 4: "memskel(two-block)"}


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 238000
    lib = _lib.load()
    fn = lib.rs_debug_ln
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 9
    H = 768
    dev = torch.device("cuda", 0)
    x32 = torch.randn(rows, H, device=dev)
    st = torch.zeros(rows, 2, device=dev)
    st[:, 1] = 1.0
    st1 = st.clone()
    o1 = (torch.randn(rows, H, device=dev) * 0.1).half()
    o2 = (torch.randn(rows, H, device=dev) * 0.1).half()
    g = torch.ones(H, device=dev)
    b = torch.zeros(H, device=dev)
    y = torch.empty(rows, H, device=dev, dtype=torch.half)
    s = torch.cuda.current_stream().cuda_stream
    p = lambda t: t.data_ptr()
    for rnd in range(2):
        for k in (0, 1, 2, 3, 4):
            call = lambda: fn(k, rows, p(x32), p(st), p(st1), p(o1), p(o2), p(g), p(b), p(y), s)
            assert call() == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                call()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 10
            print(f"round {rnd} {NAMES[k]:24s} {ms * 1e3:8.1f} us  {BYTES[k] * rows / ms / 1e6:7.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
