"""Does a scoring call on the current stream run beside rs_debug_occupy's kernel on another stream?
Times score() with n CUs held for 3 s, for n = 0, n_cu - 16, n_cu - 3, n_cu - 2."""
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import __graft_entry__  # noqa: E402

__graft_entry__._import_pkg()
from asr_rescoring_amd import _lib, data as D  # noqa: E402
from asr_rescoring_amd.scorer import PLLScorer  # noqa: E402
from asr_rescoring_amd.weights import BERT_BASE, make_weights  # noqa: E402

lib = _lib.load()
occ = lib.rs_debug_occupy
occ.restype = ctypes.c_int
occ.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
nb = D.synthetic_nbest(2, 6, seed=23, vocab=BERT_BASE.vocab, len_lo=10, len_hi=24)
s = PLLScorer(make_weights(BERT_BASE, seed=1234), BERT_BASE, device=0, max_rows=32768, precision="fp16x3")
base = s.score(nb)
n_cu = torch.cuda.get_device_properties(0).multi_processor_count
side = torch.cuda.Stream()
print("current stream", torch.cuda.current_stream().cuda_stream, "side", side.cuda_stream, flush=True)
out = torch.zeros(4096, dtype=torch.int32, device="cuda")
for gang in ("xcd", "ticket"):
    os.environ["RS_LNGANG"] = gang
    for held in (0, n_cu - 16, n_cu - 3, n_cu - 2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if held:
            assert occ(held, 3_000_000, out.data_ptr(), side.cuda_stream) == 0
        t1 = time.perf_counter()
        err = None
        try:
            got = s.score(nb)
            same = bool(np.array_equal(got, base))
        except Exception as e:  # noqa: BLE001
            err, same = str(e)[:80], None
        t2 = time.perf_counter()
        side.synchronize()
        t3 = time.perf_counter()
        spins = out[:held].cpu().numpy() if held else None
        print(f"{gang:6s} held {held:3d}: score {t2 - t1:.3f} s, occupier done at {t3 - t0:.3f} s, bitwise {same}, "
              f"error {err}, occupier spins min/max {None if spins is None else (int(spins.min()), int(spins.max()))}",
              flush=True)
s.close()
