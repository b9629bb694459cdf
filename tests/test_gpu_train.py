"""GPU parity of the native trainers (train_api.hip, k_train.hip).

Two references:
  * the reference's own training loops (fixtures F6/F7, tests/golden/make_golden_train.py:
    RescoreBert/main.py:82-229 for MD / MD_MWER / MD_MWED and MLM_PLL/main.py:73-161, two
    epochs each): epoch and dev losses, dev scores, every parameter update;
  * torch autograd + torch.optim.AdamW on the same expressions (oracle/train_ref.py) for the
    gradients of single steps.

Tolerances (fp32 on both sides, different summation orders): gradients within 2e-4 of the
reference gradient's norm per tensor; losses and scores within 1e-4 relative; parameter
updates after two epochs within 2e-2 of the update's norm (Adam normalises every element to
an lr-sized step, so near-zero gradients amplify rounding)."""
import numpy as np
import pytest
import torch

from asr_rescoring_amd import data as D
from asr_rescoring_amd.weights import BERT_TINY, make_weights

pytestmark = pytest.mark.gpu


def _batch(seed, n_utt=3, n_best=4, len_hi=20):
    nb = D.synthetic_nbest(n_utt, n_best, seed=seed, vocab=BERT_TINY.vocab, len_lo=1, len_hi=len_hi)
    rng = np.random.default_rng(seed)
    target = rng.normal(-1.0, 1.0, nb.n_hyp).astype(np.float32)
    cer = (rng.integers(0, 5, nb.n_hyp) / 10.0).astype(np.float32)
    seqs = [nb.tokens[nb.hyp_off[h]:nb.hyp_off[h + 1]].tolist() for h in range(nb.n_hyp)]
    return nb, seqs, target, nb.am.astype(np.float32), cer


def _weights(seed=1):
    return make_weights(BERT_TINY, seed=seed, with_cls_linear=True, with_pooler=True)


@pytest.mark.parametrize("method", ["MD", "MD_MWER", "MD_MWED"])
def test_gradients_match_autograd(method):
    from asr_rescoring_amd.train import RescoreBertTrainer
    from oracle.train_ref import TorchTrainer
    w = _weights()
    nb, seqs, target, am, cer = _batch(3)
    tr = RescoreBertTrainer(w, BERT_TINY, method=method, md_loss_weight=0.5)
    ref = TorchTrainer(w, BERT_TINY)
    try:
        loss, sc = tr.step(nb.tokens, nb.hyp_off, nb.utt_off, target, am, cer, update=False)
        rloss, rsc = ref.step(seqs, target, am, cer, n_best=4, method=method, md_loss_weight=0.5, update=False)
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
        # the loss-only pass (the reference's dev loss) gives the same loss and scores
        l2, sc2 = tr.step(nb.tokens, nb.hyp_off, nb.utt_off, target, am, cer, update="loss")
        assert l2 == loss and np.array_equal(sc2, sc)
    finally:
        tr.close()


@pytest.mark.parametrize("method", ["MD", "MD_MWER", "MD_MWED"])
def test_rescorebert_training_matches_reference_run(method):
    """Two epochs of the reference's RescoreBert/main.py training loop (F6): epoch losses, dev
    losses, dev scores after training and every parameter update."""
    from asr_rescoring_amd.train import RescoreBertTrainer, reference_groups, rescorebert_epoch
    from train_fixtures import check_updates, rb_fixture
    w, trd, dvd, hp, g = rb_fixture(method)
    tr = RescoreBertTrainer(w, BERT_TINY, method=method, md_loss_weight=hp["md_loss_weight"], lr=hp["lr"])
    try:
        before = {k: tr.tensor(k) for k in tr.shapes}
        tl, dl = [], []
        for _ in range(2):
            tr.reset_optimizer()
            tl.append(rescorebert_epoch(tr, trd["tokens"], trd["hyp_off"], trd["pll"], trd["am"], trd["cer"],
                                        hp["batch_size"], hp["n_best"], update=True))
            dl.append(rescorebert_epoch(tr, dvd["tokens"], dvd["hyp_off"], dvd["pll"], dvd["am"], dvd["cer"],
                                        hp["batch_size"], hp["n_best"], update="loss"))
        np.testing.assert_allclose(tl, g["train_loss"], rtol=1e-4)
        np.testing.assert_allclose(dl, g["dev_loss"], rtol=1e-4)
        n = len(dvd["hyp_off"]) - 1
        _, sc = tr.step(dvd["tokens"], dvd["hyp_off"], reference_groups(n, hp["n_best"]), dvd["pll"], dvd["am"],
                        dvd["cer"], update="loss")
        np.testing.assert_allclose(sc, g["dev_scores"], rtol=1e-4, atol=1e-5)
        check_updates(g, before, {k: tr.tensor(k) for k in tr.shapes})
    finally:
        tr.close()


def test_mlm_training_matches_reference_run():
    """Two epochs of MLM_PLL/main.py's fine-tuning loop (F7): padded batches whose [PAD]
    positions are scored with label 0, dev loss, every parameter update."""
    from asr_rescoring_amd.train import MLMTrainer, mlm_epoch
    from train_fixtures import check_updates, mlm_fixture
    w, trd, dvd, hp, g = mlm_fixture()
    tr = MLMTrainer(w, BERT_TINY, lr=hp["lr"])
    try:
        before = {k: tr.tensor(k) for k in tr.shapes}
        tl, dl = [], []
        for _ in range(2):
            tr.reset_optimizer()
            tl.append(mlm_epoch(tr, trd["seqs"], trd["labels"], hp["batch_size"], update=True))
            dl.append(mlm_epoch(tr, dvd["seqs"], dvd["labels"], hp["batch_size"], update="loss"))
        np.testing.assert_allclose(tl, g["train_loss"], rtol=1e-4)
        np.testing.assert_allclose(dl, g["dev_loss"], rtol=1e-4)
        check_updates(g, before, {k: tr.tensor(k) for k in tr.shapes})
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
        tr = RescoreBertTrainer(w, BERT_TINY, method="MD_MWED", md_loss_weight=0.3, lr=5e-4)
        for step in range(2):
            nb, _, target, am, cer = _batch(20 + step, len_hi=60)
            tr.step(nb.tokens, nb.hyp_off, nb.utt_off, target, am, cer)
        _, sc = tr.step(nb.tokens, nb.hyp_off, nb.utt_off, target, am, cer, update=False)
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
    """MLM fine-tuning on padded do_job batches: loss and every gradient vs torch autograd,
    AdamW updates vs torch.optim.AdamW, checkpoint -> PLLScorer."""
    from asr_rescoring_amd.scorer import PLLScorer
    from asr_rescoring_amd.train import MLMTrainer, do_job_rows, pad_rows
    from oracle.train_ref import TorchTrainer
    w = make_weights(BERT_TINY, seed=6)
    tr = MLMTrainer(w, BERT_TINY, lr=1e-3)
    ref = TorchTrainer(w, BERT_TINY, lr=1e-3, head="mlm")
    try:
        for step in range(2):
            nb, seqs, *_ = _batch(30 + step, n_utt=2, n_best=3, len_hi=12)
            ids, off, lab = do_job_rows(seqs)
            rows = [ids[off[i]:off[i + 1]].tolist() for i in range(len(off) - 1)]
            labs = [lab[off[i]:off[i + 1]].tolist() for i in range(len(off) - 1)]
            l = tr.step(*pad_rows(rows, labs))
            rl = ref.step_mlm(rows, labs)
            assert abs(l - rl) <= 1e-4 * abs(rl), (step, l, rl)
            if step == 0:
                gn = np.sqrt(sum(float(np.sum(ref.model.w[k].grad.numpy().astype(np.float64) ** 2))
                                 for k in tr.shapes))
                for k in tr.shapes:
                    g, rg = tr.grad(k), ref.model.w[k].grad.numpy()
                    rel = np.linalg.norm(g - rg) / max(np.linalg.norm(rg), 1e-4 * gn)
                    assert rel < 2e-4, (k, rel)
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


def test_mlm_trainer_multi_step_deterministic():
    """Regression for the CE race fixed in round 1 (the label logit read after the barrier
    that precedes the in-place gradient writes): 12 padded steps, run twice, bitwise equal
    losses and parameters, every loss within 1e-4 of torch autograd."""
    from asr_rescoring_amd.train import MLMTrainer, do_job_rows, pad_rows
    from oracle.train_ref import TorchTrainer
    w = make_weights(BERT_TINY, seed=9)
    nb, seqs, *_ = _batch(50, n_utt=4, n_best=4, len_hi=10)
    ids, off, lab = do_job_rows(seqs)
    rows = [ids[off[i]:off[i + 1]].tolist() for i in range(len(off) - 1)]
    labs = [lab[off[i]:off[i + 1]].tolist() for i in range(len(off) - 1)]
    batches = [(rows[b:b + 8], labs[b:b + 8]) for b in range(0, len(rows), 8)][:12]
    runs = []
    for _ in range(2):
        tr = MLMTrainer(w, BERT_TINY, lr=1e-3)
        try:
            losses = [tr.step(*pad_rows(r, l)) for r, l in batches]
            runs.append((losses, {k: tr.tensor(k) for k in tr.shapes}))
        finally:
            tr.close()
    assert runs[0][0] == runs[1][0]
    assert all(np.array_equal(runs[0][1][k], runs[1][1][k]) for k in runs[0][1])
    ref = TorchTrainer(w, BERT_TINY, lr=1e-3, head="mlm")
    want = [ref.step_mlm(r, l) for r, l in batches]
    np.testing.assert_allclose(runs[0][0][:3], want[:3], rtol=1e-4)
    np.testing.assert_allclose(runs[0][0], want, rtol=1e-3)   # later steps: AdamW amplifies rounding
