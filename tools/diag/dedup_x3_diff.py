"""Which rows differ between RS_DEDUP=1 and 0 in the fp16x3 split-operand mode (diagnostic)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import __graft_entry__  # noqa: E402

__graft_entry__._import_pkg()
from asr_rescoring_amd import data as D  # noqa: E402
from asr_rescoring_amd.scorer import PLLScorer  # noqa: E402
from asr_rescoring_amd.weights import BERT_TINY, make_weights  # noqa: E402

w = make_weights(BERT_TINY, seed=1)
for max_rows, lh in ((512, 70), (65536, 70), (65536, 40), (512, 40)):
    nb = D.synthetic_nbest(5, 4, seed=5, vocab=BERT_TINY.vocab, len_lo=1, len_hi=lh)
    s = PLLScorer(w, BERT_TINY, device=0, max_rows=max_rows, precision="fp16x3")
    out = {}
    for dd in ("1", "0", "1"):
        os.environ["RS_DEDUP"] = dd
        out.setdefault(dd, []).append(s.score(nb))
    s.close()
    a, b, a2 = out["1"][0], out["0"][0], out["1"][1]
    lens = np.diff(nb.hyp_off)
    bad = np.nonzero(a != b)[0]
    print(f"max_rows {max_rows} len_hi {lh}: dedup deterministic {np.array_equal(a, a2)}; "
          f"{len(bad)}/{len(a)} hyps differ; lens of differing {lens[bad].tolist()}; "
          f"max rel {np.max(np.abs(a - b) / np.abs(b)):.2e}", flush=True)
