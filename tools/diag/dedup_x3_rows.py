"""Per masked row: which (hypothesis, position) rows differ between RS_DEDUP=1 and 0 in the
fp16x3 split-operand mode (diagnostic)."""
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
nb = D.synthetic_nbest(5, 4, seed=5, vocab=BERT_TINY.vocab, len_lo=1, len_hi=40)
s = PLLScorer(w, BERT_TINY, device=0, max_rows=65536, precision="fp16x3")
res = {}
for env in ({"RS_DEDUP": "1"}, {"RS_DEDUP": "0"}, {"RS_DEDUP": "1", "RS_X3S_IMGRES": "0"}, {"RS_DEDUP": "0", "RS_X3S_IMGRES": "0"}):
    for k in ("RS_DEDUP", "RS_X3S_IMGRES"):
        os.environ.pop(k, None)
    os.environ.update(env)
    _, rows = s.score_nbest(nb.tokens, nb.hyp_off, return_rows=True)
    res[tuple(sorted(env.items()))] = rows.cpu().numpy()
s.close()
keys = list(res)
a, b = res[keys[0]], res[keys[1]]
lens = np.diff(nb.hyp_off) - 2
off = np.concatenate([[0], np.cumsum(lens)])
for h in range(len(lens)):
    d = np.nonzero(a[off[h]:off[h + 1]] != b[off[h]:off[h + 1]])[0]
    if len(d):
        print(f"hyp {h} (L={lens[h]}): differing masked positions {d.tolist()}")
print("imgres=0 dedup on vs off equal:", np.array_equal(res[keys[2]], res[keys[3]]))
print("dedup=0: imgres 1 vs 0 max rel", float(np.max(np.abs(res[keys[1]] - res[keys[3]]) / np.abs(res[keys[3]]))))
