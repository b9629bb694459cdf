"""Shared by the CPU oracle tests and the GPU trainer tests: the F6/F7 training fixtures
(tests/golden/make_golden_train.py — the reference's own training loops, two epochs) and the
comparison of a trained parameter set against their update sketches."""
import os

import numpy as np

from asr_rescoring_amd.weights import BERT_TINY, make_weights, weights_digest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
METHODS = ("MD", "MD_MWER", "MD_MWED")


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def rb_fixture(method):
    """(weights, train dict, dev dict, hyper-parameters, fixture) of train_rb_<method>.npz."""
    g = load(f"train_rb_{method}.npz")
    w = make_weights(BERT_TINY, seed=int(g["weight_seed"]), with_cls_linear=True, with_pooler=True)
    assert weights_digest(w) == str(g["digest"])

    def split(p):
        tok, off = g[p + "tokens"], g[p + "hyp_off"]
        return dict(tokens=tok, hyp_off=off, seqs=[tok[off[h]:off[h + 1]].tolist() for h in range(len(off) - 1)],
                    pll=g[p + "pll"], am=g[p + "am"], cer=g[p + "cer"])
    hp = dict(n_best=int(g["n_best"]), batch_size=int(g["batch_size"]), md_loss_weight=float(g["md_loss_weight"]),
              lr=float(g["lr"]))
    return w, split("tr_"), split("dv_"), hp, g


def mlm_fixture():
    g = load("train_mlm.npz")
    w = make_weights(BERT_TINY, seed=int(g["weight_seed"]))
    assert weights_digest(w) == str(g["digest"])

    def split(p):
        ids, lab, off = g[p + "ids"], g[p + "labels"], g[p + "off"]
        n = len(off) - 1
        return dict(seqs=[ids[off[i]:off[i + 1]].tolist() for i in range(n)],
                    labels=[lab[off[i]:off[i + 1]].tolist() for i in range(n)])
    return w, split("tr_"), split("dv_"), dict(batch_size=int(g["batch_size"]), lr=float(g["lr"])), g


def check_updates(g, before, after, rel=2e-2):
    """Every parameter's update (after - before) against the fixture's sketch: L2 norm and the
    probe dot within ``rel`` of the reference update's norm, whole small tensors elementwise
    within ``rel`` of their norm.  Parameters the fixture has but ``after`` lacks (the unused
    pooler) must not have moved in the reference either.  ``attention.self.key.bias`` is
    skipped: its gradient is exactly zero in exact arithmetic (softmax shift invariance), so
    each side's AdamW turns its own rounding noise into noise-signed lr-sized steps."""
    keys = sorted(k[3:] for k in g.files if k.startswith("sk/"))
    worst = {}
    for i, k in enumerate(keys):
        s = g["sk/" + k]
        if k.endswith("attention.self.key.bias"):
            continue
        if k not in after:
            assert s[1] == 0.0, (k, s)
            continue
        d = (after[k].astype(np.float64) - before[k].astype(np.float64)).ravel()
        r = np.random.Generator(np.random.PCG64(1000 + i)).standard_normal(d.size)
        nrm = max(s[1], 1e-12)
        e = max(abs(np.linalg.norm(d) - s[1]), abs(float(d @ r) - s[2])) / nrm
        if "full/" + k in g.files:
            e = max(e, float(np.abs(d - g["full/" + k]).max()) / nrm)
        worst[k] = e
    bad = {k: v for k, v in worst.items() if v > rel}
    assert not bad, sorted(bad.items(), key=lambda kv: -kv[1])[:6]
    return worst
