"""Scores of two library builds compared BITWISE on the same inputs (one process per build:
RS_LIBRESCORE selects the library).  Usage:
    bitwise_ab.py LIB_A LIB_B OUTDIR     (parent: runs both, compares, prints one JSON line;
                                          LIB@VAR=VALUE,...: that library under env switches)
Inputs: the fp16x3 golden tokens (F1), 40 C3 utterances x N=50, 150 C4 utterances x N=100 at the
alfred real lengths; bert-base random init seed 1234, fp16x3, default kernels."""
import json
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def run_one(out):
    import torch
    import __graft_entry__
    __graft_entry__._import_pkg()
    from asr_rescoring_amd import data as D
    from asr_rescoring_amd.scorer import PLLScorer
    from asr_rescoring_amd.weights import BERT_BASE, make_weights
    w = make_weights(BERT_BASE, seed=1234)
    s = PLLScorer(w, BERT_BASE, device=0, max_rows=262144, precision="fp16x3")
    res = {}
    g = np.load(os.path.join(REPO, "tests", "golden", "pll_base.npz"))
    pll, rows = s.score_nbest(g["tokens"], g["hyp_off"], return_rows=True)
    res["f1_pll"], res["f1_rows"] = pll.cpu().numpy(), rows.cpu().numpy()
    nb = D.synthetic_nbest(40, 50, seed=1, hard=True)
    res["c3_pll"] = s.score_nbest(nb.tokens, nb.hyp_off).cpu().numpy()
    lc = json.load(open(os.path.join(REPO, "tests", "golden", "alfred_test_lengths.json")))["length_counts"]
    lengths = np.repeat(np.arange(len(lc)), lc).astype(np.int64)
    nb4 = D.synthetic_nbest(150, 100, seed=1, lengths=lengths, hard=True)
    res["c4_pll"] = s.score_nbest(nb4.tokens, nb4.hyp_off).cpu().numpy()
    torch.cuda.synchronize()
    s.close()
    np.savez(out, **res)


if __name__ == "__main__":
    if sys.argv[1] == "--one":
        run_one(sys.argv[2])
        sys.exit(0)
    la, lb, od = sys.argv[1:4]
    os.makedirs(od, exist_ok=True)
    outs = []
    for tag, spec in (("a", la), ("b", lb)):
        # LIB or LIB@VAR=VALUE,...: the same library under other environment switches
        lib, _, envs = spec.partition("@")
        o = os.path.join(od, f"scores_{tag}.npz")
        env = dict(os.environ, RS_LIBRESCORE=os.path.abspath(lib))
        env.update(dict(kv.split("=", 1) for kv in envs.split(",") if kv))
        subprocess.run([sys.executable, os.path.abspath(__file__), "--one", o], env=env, check=True, timeout=600)
        outs.append(np.load(o))
    rec = {"lib_a": la, "lib_b": lb}
    for k in outs[0].files:
        a, b = outs[0][k], outs[1][k]
        rec[k] = {"n": int(a.size), "bitwise_equal": bool(np.array_equal(a.view(np.uint8), b.view(np.uint8))),
                  "max_rel_diff": float(np.max(np.abs(a - b) / np.maximum(np.abs(a), 1e-30)))}
    print(json.dumps(rec))
