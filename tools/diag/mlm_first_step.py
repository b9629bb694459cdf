"""Regression check: the MLM trainer's first-step loss vs the torch reference, in several construction orders (run it in a few fresh processes: the tr_ce race it guards against was intermittent)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import __graft_entry__  # noqa: E402

__graft_entry__._import_pkg()
from asr_rescoring_amd import data as D  # noqa: E402
from asr_rescoring_amd.train import MLMTrainer, do_job_rows  # noqa: E402
from asr_rescoring_amd.weights import BERT_TINY, make_weights  # noqa: E402
from oracle.train_ref import TorchTrainer  # noqa: E402


def batch(seed):
    nb = D.synthetic_nbest(2, 3, seed=seed, vocab=BERT_TINY.vocab, len_lo=1, len_hi=12)
    seqs = [nb.tokens[nb.hyp_off[h]:nb.hyp_off[h + 1]].tolist() for h in range(nb.n_hyp)]
    return do_job_rows(seqs)


for variant in ("test-order", "test-order-again", "ref-first", "no-ref"):
    w = make_weights(BERT_TINY, seed=6)
    ids, off, lab = batch(30)
    if variant == "ref-first":
        ref = TorchTrainer(w, BERT_TINY, lr=1e-3, head="mlm")
        tr = MLMTrainer(w, BERT_TINY, lr=1e-3)
    else:
        tr = MLMTrainer(w, BERT_TINY, lr=1e-3)
        ref = TorchTrainer(w, BERT_TINY, lr=1e-3, head="mlm") if variant != "no-ref" else None
    l = tr.step(ids, off, lab)
    rl = ref.step_mlm(ids, off, lab) if ref else float("nan")
    tr.close()
    print(f"{variant}: trainer {l} ref {rl}", flush=True)
