"""GPU parity of the native RescoreBert trainer (train_api.hip, k_train.hip) against torch
autograd + torch.optim.AdamW on the same loss (oracle/train_ref.py).

Tolerances (fp32 on both sides, different summation orders): gradients within 2e-4 of the
reference gradient's norm per tensor; parameters after AdamW steps within 1e-5 absolute
(updates are lr-sized); losses and scores within 1e-4 relative."""
import numpy as np
import pytest
import torch

from asr_rescoring_amd import data as D
from asr_rescoring_amd.weights import BERT_TINY, make_weights

pytestmark = pytest.mark.gpu


def _batch(seed, n_utt=3, n_best=4, len_hi=20):
    nb = D.synthetic_nbest(n_utt, n_best, seed=seed, vocab=BERT_TINY.vocab, len_lo=1, len_hi=len_hi)
    rng = np.random.default_rng(seed)
    target = -np.abs(rng.normal(20, 5, nb.n_hyp)).astype(np.float32)
    err = rng.integers(0, 5, nb.n_hyp).astype(np.float32)
    seqs = [nb.tokens[nb.hyp_off[h]:nb.hyp_off[h + 1]].tolist() for h in range(nb.n_hyp)]
    return nb, seqs, target, nb.am.astype(np.float32), err


def _weights(seed=1):
    return make_weights(BERT_TINY, seed=seed, with_cls_linear=True, with_pooler=True)


@pytest.mark.parametrize("kind", ["MD", "MD_MWER", "MD_MWED"])
def test_gradients_match_autograd(kind):
    from asr_rescoring_amd.train import RescoreBertTrainer
    from oracle.train_ref import TorchTrainer
    w = _weights()
    nb, seqs, target, am, err = _batch(3)
    tr = RescoreBertTrainer(w, BERT_TINY, loss=kind, lam=0.5)
    ref = TorchTrainer(w, BERT_TINY)
    try:
        loss, sc = tr.step(nb.tokens, nb.hyp_off, nb.utt_off, target, am, err, update=False)
        rloss, rsc = ref.step(seqs, nb.utt_off, target, am, err, kind=kind, lam=0.5, update=False)
        assert abs(loss - rloss) <= 1e-4 * abs(rloss)
        assert np.abs(sc - rsc).max() <= 1e-4 * np.abs(rsc).max()
        # relative to the tensor's own gradient norm, floored at 1e-4 of the global norm:
        # attention.self.key.bias has an exactly-zero gradient (softmax shift invariance),
        # so both sides hold rounding noise there
        gnorm = np.sqrt(sum(float(np.sum(ref.grad(k).astype(np.float64) ** 2)) for k in tr.shapes))
        for k in tr.shapes:
            g, rg = tr.grad(k), ref.grad(k)
            rel = np.linalg.norm(g - rg) / max(np.linalg.norm(rg), 1e-4 * gnorm)
            assert rel < 2e-4, (k, rel, np.linalg.norm(rg))
    finally:
        tr.close()


def test_adamw_steps_match_torch():
    from asr_rescoring_amd.train import RescoreBertTrainer
    from oracle.train_ref import TorchTrainer
    w = _weights(2)
    tr = RescoreBertTrainer(w, BERT_TINY, loss="MD_MWER", lam=1.0, lr=1e-3)
    ref = TorchTrainer(w, BERT_TINY, lr=1e-3)
    try:
        for step in range(3):
            nb, seqs, target, am, err = _batch(10 + step)
            l, _ = tr.step(nb.tokens, nb.hyp_off, nb.utt_off, target, am, err)
            rl, _ = ref.step(seqs, nb.utt_off, target, am, err, kind="MD_MWER", lam=1.0)
            assert abs(l - rl) <= 1e-4 * abs(rl), (step, l, rl)
        # Adam normalises every gradient element to an ~lr-sized step, so elements whose
        # gradient is rounding noise (key.bias entirely, a few others) move by noise-signed
        # lr steps on either side: compare the whole update per tensor instead
        worst = {}
        for k in tr.shapes:
            if k.endswith("attention.self.key.bias"):
                continue
            d, dr = tr.tensor(k) - w[k], ref.tensor(k) - w[k]
            worst[k] = float(np.linalg.norm(d - dr) / max(np.linalg.norm(dr), 1e-12))
        assert max(worst.values()) < 2e-2, sorted(worst.items(), key=lambda kv: -kv[1])[:4]
    finally:
        tr.close()


def test_trained_checkpoint_feeds_the_scorer_and_is_deterministic():
    """state_dict() -> RescoreBertScorer reproduces the trainer's forward scores; two trainers
    on the same data end bitwise equal."""
    from asr_rescoring_amd.scorer import RescoreBertScorer
    from asr_rescoring_amd.train import RescoreBertTrainer
    w = _weights(4)
    out = []
    for _ in range(2):
        tr = RescoreBertTrainer(w, BERT_TINY, loss="MD_MWED", lam=0.3, lr=5e-4)
        for step in range(2):
            nb, _, target, am, err = _batch(20 + step, len_hi=60)
            tr.step(nb.tokens, nb.hyp_off, nb.utt_off, target, am, err)
        _, sc = tr.step(nb.tokens, nb.hyp_off, nb.utt_off, target, am, err, update=False)
        out.append((tr.state_dict(), sc))
        tr.close()
    (sd, sc), (sd2, sc2) = out
    assert all(np.array_equal(sd[k], sd2[k]) for k in sd) and np.array_equal(sc, sc2)
    scorer = RescoreBertScorer(sd, BERT_TINY, device=0, precision="fp16x3")
    try:
        got = scorer.score_nbest(nb.tokens, nb.hyp_off).cpu().numpy()
    finally:
        scorer.close()
    assert np.abs(got - sc).max() <= 1e-4 * max(1.0, np.abs(sc).max())


def test_mlm_finetune_matches_autograd_and_feeds_the_pll_scorer():
    """MLM fine-tuning (MLM_PLL/main.py:117-161) on do_job rows: loss and every gradient vs
    torch autograd, AdamW updates vs torch.optim.AdamW, checkpoint -> PLLScorer."""
    from asr_rescoring_amd.scorer import PLLScorer
    from asr_rescoring_amd.train import MLMTrainer, do_job_rows
    from oracle.train_ref import TorchTrainer
    w = make_weights(BERT_TINY, seed=6)
    tr = MLMTrainer(w, BERT_TINY, lr=1e-3)
    ref = TorchTrainer(w, BERT_TINY, lr=1e-3, head="mlm")
    try:
        for step in range(2):
            nb, seqs, *_ = _batch(30 + step, n_utt=2, n_best=3, len_hi=12)
            ids, off, lab = do_job_rows(seqs)
            l = tr.step(ids, off, lab)
            rl = ref.step_mlm(ids, off, lab)
            assert abs(l - rl) <= 1e-4 * abs(rl), (step, l, rl)
            if step == 0:
                gn = np.sqrt(sum(float(np.sum(ref.model.w[k].grad.numpy().astype(np.float64) ** 2))
                                 for k in tr.shapes))
                for k in tr.shapes:
                    g, rg = tr.grad(k), ref.model.w[k].grad.numpy()
                    rel = np.linalg.norm(g - rg) / max(np.linalg.norm(rg), 1e-4 * gn)
                    assert rel < 2e-4, (k, rel)
        worst = {}
        for k in tr.shapes:
            if k.endswith("attention.self.key.bias"):
                continue
            d, dr = tr.tensor(k) - w[k], ref.tensor(k) - w[k]
            worst[k] = float(np.linalg.norm(d - dr) / max(np.linalg.norm(dr), 1e-12))
        assert max(worst.values()) < 2e-2, sorted(worst.items(), key=lambda kv: -kv[1])[:4]
        sd = tr.state_dict()
    finally:
        tr.close()
    nb, seqs, *_ = _batch(40, n_utt=2, n_best=3, len_hi=12)
    sc = PLLScorer(sd, BERT_TINY, device=0, precision="fp16x3")
    try:
        got = sc.score(nb)
    finally:
        sc.close()
    from oracle.bert_ref import TorchBert, pll_reference_pattern
    _, want = pll_reference_pattern(TorchBert(sd, BERT_TINY), nb.tokens, nb.hyp_off, full_head=False)
    assert (np.abs(got - want) / np.abs(want)).max() < 1e-3
