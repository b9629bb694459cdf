"""In-process A/B of launch switches that are read per call (RS_LNGANG, RS_CHUNK_ALIGN, ...)
on the bench's C3 workload: one scorer, one synthetic set, the configurations interleaved
round by round; prints masked forwards/s per configuration (median over rounds) and whether
every configuration's PLL scores are bitwise equal to the first one's.

Usage: python tools/env_ab.py UTTS ROUNDS 'A=1' 'A=2;B=x' ''   ('' = no switch set)
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__  # noqa: E402

__graft_entry__._import_pkg()
from asr_rescoring_amd import data as D  # noqa: E402
from asr_rescoring_amd.scorer import PLLScorer  # noqa: E402
from asr_rescoring_amd.weights import BERT_BASE, make_weights  # noqa: E402


def parse(cfg):
    out = {}
    for kv in filter(None, cfg.split(";")):
        k, v = kv.split("=", 1)
        out[k] = v
    return out


def main():
    utts, rounds = int(sys.argv[1]), int(sys.argv[2])
    cfgs = sys.argv[3:] or [""]
    nb = D.synthetic_nbest(utts, 50, seed=1, hard=True)
    scorer = PLLScorer(make_weights(BERT_BASE, seed=1234), BERT_BASE, device=0, max_rows=262144)
    tok = torch.from_numpy(nb.tokens).cuda()
    n_fwd = nb.n_forwards()
    keys = sorted({k for c in cfgs for k in parse(c)})
    times = {c: [] for c in cfgs}
    ref, same = None, {c: True for c in cfgs}
    for r in range(rounds):
        for c in cfgs:
            for k in keys:
                os.environ.pop(k, None)
            os.environ.update(parse(c))
            scorer.score_nbest(tok, nb.hyp_off)                  # warm (per-call switches applied)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            lm = scorer.score_nbest(tok, nb.hyp_off)
            torch.cuda.synchronize()
            times[c].append(time.perf_counter() - t0)
            v = lm.cpu().numpy()
            if ref is None:
                ref = v
            same[c] = same[c] and np.array_equal(v, ref)
        print(f"round {r}: " + "  ".join(f"[{c or 'base'}] {n_fwd / times[c][-1]:.0f}" for c in cfgs), flush=True)
    for c in cfgs:
        med = sorted(times[c])[len(times[c]) // 2]
        print(f"{c or 'base':40s} {n_fwd / med:9.0f} masked fwd/s  {med * 1e3:8.1f} ms  bitwise={same[c]}", flush=True)
    scorer.close()


if __name__ == "__main__":
    main()
