"""Where do workgroups go when some CUs are held?  Another process holds `held` CUs for 2 s
(rs_debug_occupy, one 160 KiB-LDS workgroup per CU); this process then times, on its own stream,
  lds36  — 36 workgroups of the same 160 KiB-LDS kernel for 1 ms (placement recorded),
  x3s    — one split-operand GEMM (rs_debug_gemm cfg 32, 3072 x 768 x 768: 36 tiles),
  blas   — torch fp16 matmul of the same shape (a library GEMM),
and prints the occupier's and the probe's placement per (XCC, SE, SH)."""
import collections
import ctypes
import json
import os
import subprocess
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import __graft_entry__  # noqa: E402

__graft_entry__._import_pkg()
from asr_rescoring_amd import _lib  # noqa: E402

OCC = r"""
import ctypes, json, sys, time
import torch
sys.path.insert(0, {repo!r})
import __graft_entry__
__graft_entry__._import_pkg()
from asr_rescoring_amd import _lib
fn = _lib.load().rs_debug_occupy
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
out = torch.zeros(4096, dtype=torch.int32, device="cuda")
torch.cuda.synchronize()
for line in sys.stdin:
    held = int(line)
    if held < 0:
        break
    assert fn(held, 2_000_000, out.data_ptr(), 0) == 0
    time.sleep(0.05)
    print("ready", flush=True)
    torch.cuda.synchronize()
    print(json.dumps(out[held:2 * held].cpu().tolist()), flush=True)
"""


def where(words):
    c = collections.Counter()
    for w in words:
        w &= 0xffffffff
        xcc, hw = w >> 24, w & 0xffffff
        se, sh, cu = (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 15
        c[(xcc, se, sh)] += 1
    return dict(sorted(c.items()))


lib = _lib.load()
occ = lib.rs_debug_occupy
occ.restype = ctypes.c_int
occ.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
dg = lib.rs_debug_gemm
dg.restype = ctypes.c_int
dg.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_int] * 3 + [ctypes.c_void_p]
M, N, K = 3072, 768, 768
a = (torch.randn(M, 2 * K, device="cuda") * 0.1).half()
w = (torch.randn(N, 2 * K, device="cuda") * 0.1).half()
bias = torch.zeros(N, device="cuda")
c32 = torch.empty(M, N, device="cuda")
a16, w16 = a[:, :K].contiguous(), w[:, :K].contiguous()
out = torch.zeros(4096, dtype=torch.int32, device="cuda")
mine = torch.cuda.Stream()
torch.cuda.synchronize()
p = subprocess.Popen([sys.executable, "-c", OCC.format(repo=REPO)], stdin=subprocess.PIPE,
                     stdout=subprocess.PIPE, text=True)


def run(what):
    if what == "lds36":
        assert occ(36, 1000, out.data_ptr(), mine.cuda_stream) == 0
    elif what == "x3s":
        assert dg(32, 0, a.data_ptr(), w.data_ptr(), bias.data_ptr(), c32.data_ptr(), M, N, K, mine.cuda_stream) == 0
    else:
        torch.matmul(a16, w16.t())


with torch.cuda.stream(mine):
    for what in ("lds36", "x3s", "blas"):
        run(what)
mine.synchronize()
n_cu = torch.cuda.get_device_properties(0).multi_processor_count
print(f"n_cu {n_cu}", flush=True)
for held in (0, 128, 192, 216, 224, 232, 240, 248):
    for what in ("lds36", "x3s", "blas"):
        if held:
            p.stdin.write(f"{held}\n")
            p.stdin.flush()
            assert p.stdout.readline().strip() == "ready"
        t0 = time.perf_counter()
        with torch.cuda.stream(mine):
            run(what)
        mine.synchronize()
        dt = time.perf_counter() - t0
        extra = ""
        if what == "lds36":
            extra = " probe at " + json.dumps({str(k): v for k, v in where(out[36:72].cpu().tolist()).items()})
        held_at = where(json.loads(p.stdout.readline())) if held else {}
        print(f"held {held:3d} {what:5s} {dt * 1e3:8.2f} ms{extra}", flush=True)
        if held and what == "lds36":
            print("   occupier at " + json.dumps({str(k): v for k, v in held_at.items()}), flush=True)
p.stdin.write("-1\n")
p.stdin.flush()
p.wait(timeout=60)
