"""Which work runs beside a kernel that holds CUs?  An occupier (rs_debug_occupy: one 160 KiB-LDS
workgroup per CU for 2 s) runs in another process ("proc") or on a side stream of this process
("stream"); meanwhile this process times, on its own stream:
  tiny   — a 1-workgroup elementwise kernel,
  wide   — a 64 Mi-element elementwise kernel (workgroups on every XCD),
  score  — one PLL scoring call of a small N-best list (the LayerNorm-gang GEMMs inside).
A time near 2 s means the work waited for the occupier."""
import ctypes
import os
import subprocess
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import __graft_entry__  # noqa: E402

__graft_entry__._import_pkg()
from asr_rescoring_amd import _lib, data as D  # noqa: E402
from asr_rescoring_amd.scorer import PLLScorer  # noqa: E402
from asr_rescoring_amd.weights import BERT_BASE, make_weights  # noqa: E402

OCC = r"""
import ctypes, sys, time
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
    print("done", flush=True)
"""

lib = _lib.load()
occ = lib.rs_debug_occupy
occ.restype = ctypes.c_int
occ.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
nb = D.synthetic_nbest(2, 6, seed=23, vocab=BERT_BASE.vocab, len_lo=10, len_hi=24)
s = PLLScorer(make_weights(BERT_BASE, seed=1234), BERT_BASE, device=0, max_rows=32768, precision="fp16x3")
base = s.score(nb)
n_cu = torch.cuda.get_device_properties(0).multi_processor_count
mine = torch.cuda.Stream()
side = torch.cuda.Stream()
out = torch.zeros(4096, dtype=torch.int32, device="cuda")
x1 = torch.ones(256, device="cuda")
x2 = torch.ones(1 << 26, device="cuda")
torch.cuda.synchronize()
p = subprocess.Popen([sys.executable, "-c", OCC.format(repo=REPO)], stdin=subprocess.PIPE,
                     stdout=subprocess.PIPE, text=True)


def timed(fn):
    t0 = time.perf_counter()
    with torch.cuda.stream(mine):
        fn()
    mine.synchronize()
    return time.perf_counter() - t0


def tiny():
    x1.add_(1)


def wide():
    x2.add_(1)


res = {}


def score():
    res["same"] = bool(np.array_equal(s.score(nb), base))


print(f"n_cu {n_cu}", flush=True)
for mode in ("proc", "stream"):
    for held in (8, 64, 128, 192, 240, 248, 253):
        for what, fn in (("tiny", tiny), ("wide", wide), ("score", score)):
            if mode == "proc":
                p.stdin.write(f"{held}\n")
                p.stdin.flush()
                assert p.stdout.readline().strip() == "ready"
            else:
                torch.cuda.synchronize()
                assert occ(held, 2_000_000, out.data_ptr(), side.cuda_stream) == 0
                time.sleep(0.05)
            err = None
            try:
                dt = timed(fn)
            except Exception as e:  # noqa: BLE001
                dt, err = float("nan"), str(e)[:60]
            if mode == "proc":
                assert p.stdout.readline().strip() == "done"
            else:
                side.synchronize()
            print(f"{mode:6s} held {held:3d} {what:5s} {dt:.3f} s"
                  + (f" bitwise {res.get('same')}" if what == "score" and err is None else "")
                  + (f" error {err}" if err else ""), flush=True)
            res.clear()
p.stdin.write("-1\n")
p.stdin.flush()
p.wait(timeout=60)
s.close()
