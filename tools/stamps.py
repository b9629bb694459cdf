"""Phase shares of the split-operand GEMM tiles from the stamp build (rs_debug_stamps): one
scoring pass of the C3 workload (U utterances x N=50) with every split-operand launch running its
stamp build; prints, per kernel instance, the mean cycles per tile of each phase (kstep0: the tile's
first K-step, from the end of the previous tile's stores; kloop: the rest) (wave 0 of each
workgroup; s_memtime ticks) and its share.  The stamp build's fences forbid overlaps the production
kernel has: read the SHARES, not the absolute time.
Usage: python tools/stamps.py [U] [RS_LNGANG]"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# the timing-diagnostic build (build.py --diag): the wrong-results GEMM variants / the stamp build
os.environ.setdefault("RS_LIBRESCORE", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                    "asr-rescoring_amd", "librescore_diag.so"))
import __graft_entry__  # noqa: E402

__graft_entry__._import_pkg()
from asr_rescoring_amd import _lib, data as D  # noqa: E402
from asr_rescoring_amd.scorer import PLLScorer  # noqa: E402
from asr_rescoring_amd.weights import BERT_BASE, make_weights  # noqa: E402

PHASES = ["kloop", "bias+next_stage", "residual", "stats+publish", "poll", "ln_apply", "stores"]
INST = ["qkv/fp32", "ffn1/gelu", "oproj+LN", "ffn2+LN"]


def main():
    U = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    if len(sys.argv) > 2:
        os.environ["RS_LNGANG"] = sys.argv[2]
    lib = _lib.load()
    fn = lib.rs_debug_stamps
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int, ctypes.c_void_p]
    nb = D.synthetic_nbest(U, 50, seed=1, hard=True)
    sc = PLLScorer(make_weights(BERT_BASE, seed=1234), BERT_BASE, device=0, max_rows=262144)
    tok = torch.from_numpy(nb.tokens).cuda()
    sc.score_nbest(tok, nb.hyp_off)                  # warm
    torch.cuda.synchronize()
    assert fn(1, None) == 0
    sc.score_nbest(tok, nb.hyp_off)
    torch.cuda.synchronize()
    buf = np.zeros(4 * 256 * 16, np.uint64)
    assert fn(0, buf.ctypes.data) == 0
    st = buf.reshape(4, 256, 16).astype(np.float64)
    for i, name in enumerate(INST):
        tiles = st[i, :, 7].sum()
        if tiles == 0:
            continue
        per = st[i, :, :7].sum(axis=0) / tiles
        tot = per.sum()
        pro = st[i, :, 8].sum() / max((st[i, :, 7] > 0).sum(), 1)
        k0 = st[i, :, 9].sum() / tiles                  # K-step 0 (wait for the tile's stage 0 + first barrier)
        tot += k0
        print(f"{name:10s} tiles {int(tiles):7d}  cycles/tile {tot:9.0f}  prologue/workgroup {pro:8.0f}  "
              f"kstep0 {k0:7.0f} ({k0 / tot * 100:4.1f}%)  " +
              "  ".join(f"{p} {v:7.0f} ({v / tot * 100:4.1f}%)" for p, v in zip(PHASES, per) if v > 0), flush=True)
    sc.close()


if __name__ == "__main__":
    main()
