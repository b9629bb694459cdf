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

# the fixture-pinned mode: dropout off (the golden runs switch it off through BertConfig)
NO_DROP = dict(hidden_dropout=0.0, attn_dropout=0.0)


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
    tr = RescoreBertTrainer(w, BERT_TINY, method=method, md_loss_weight=0.5, **NO_DROP)
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


def test_gradients_match_autograd_past_the_one_pass_column_sums():
    """A batch of more than 2048 token rows: the trainer's bias / LayerNorm column sums take their
    two-stage form (k_train.hip tr_colsum, kOnePass) and the GEMM picker other tiles — gradients
    against torch autograd as above."""
    from asr_rescoring_amd.train import RescoreBertTrainer
    from oracle.train_ref import TorchTrainer
    w = _weights()
    nb, seqs, target, am, cer = _batch(5, n_utt=12, n_best=16, len_hi=30)
    assert int(nb.hyp_off[-1]) > 2048
    tr = RescoreBertTrainer(w, BERT_TINY, method="MD_MWER", md_loss_weight=0.5, **NO_DROP)
    ref = TorchTrainer(w, BERT_TINY)
    try:
        loss, sc = tr.step(nb.tokens, nb.hyp_off, nb.utt_off, target, am, cer, update=False)
        rloss, rsc = ref.step(seqs, target, am, cer, n_best=16, method="MD_MWER", md_loss_weight=0.5, update=False)
        assert abs(loss - rloss) <= 1e-4 * abs(rloss)
        assert np.abs(sc - rsc).max() <= 1e-4 * np.abs(rsc).max()
        gnorm = np.sqrt(sum(float(np.sum(ref.grad(k).astype(np.float64) ** 2)) for k in tr.shapes))
        for k in tr.shapes:
            g, rg = tr.grad(k), ref.grad(k)
            rel = np.linalg.norm(g - rg) / max(np.linalg.norm(rg), 1e-4 * gnorm)
            assert rel < 2e-4, (k, rel, np.linalg.norm(rg))
    finally:
        tr.close()


@pytest.mark.parametrize("method", ["MD", "MD_MWER", "MD_MWED"])
def test_rescorebert_training_matches_reference_run(method):
    """Two epochs of the reference's RescoreBert/main.py training loop (F6): epoch losses, dev
    losses, dev scores after training and every parameter update."""
    from asr_rescoring_amd.train import RescoreBertTrainer, reference_groups, rescorebert_epoch
    from train_fixtures import check_updates, rb_fixture
    w, trd, dvd, hp, g = rb_fixture(method)
    tr = RescoreBertTrainer(w, BERT_TINY, method=method, md_loss_weight=hp["md_loss_weight"], lr=hp["lr"], **NO_DROP)
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


def test_md_epoch_on_batches_that_do_not_reshape():
    """MD is a plain MSELoss(sum) over the batch (RescoreBert/main.py:104-110): it trains on an
    N-best set whose batches are not multiples of n_best (17 hypotheses, batches of 2 x 4 rows:
    8, 8, 1), where MD_MWER / MD_MWED's reshape(-1, n_best) would fail."""
    from asr_rescoring_amd.train import RescoreBertTrainer, rescorebert_epoch
    from oracle.train_ref import TorchTrainer, train_rescorebert
    w = _weights(5)
    nb, seqs, target, am, cer = _batch(60, n_utt=5, n_best=4)
    H = 17
    toks, hoff = nb.tokens[:nb.hyp_off[H]], nb.hyp_off[:H + 1]
    tr = RescoreBertTrainer(w, BERT_TINY, method="MD", lr=1e-3, **NO_DROP)
    ref = TorchTrainer(w, BERT_TINY, lr=1e-3)
    try:
        tr.reset_optimizer()
        tl = rescorebert_epoch(tr, toks, hoff, target[:H], am[:H], cer[:H], 2, 4, update=True)
        dl = rescorebert_epoch(tr, toks, hoff, target[:H], am[:H], cer[:H], 2, 4, update="loss")
        split = dict(seqs=seqs[:H], pll=target[:H], am=am[:H], cer=cer[:H])
        rtl, rdl = train_rescorebert(ref, split, split, 1, 2, 4, "MD", 1.0)
        np.testing.assert_allclose([tl, dl], [rtl[0], rdl[0]], rtol=1e-4)
    finally:
        tr.close()


def test_mlm_training_matches_reference_run():
    """Two epochs of MLM_PLL/main.py's fine-tuning loop (F7): padded batches whose [PAD]
    positions are scored with label 0, dev loss, every parameter update."""
    from asr_rescoring_amd.train import MLMTrainer, mlm_epoch
    from train_fixtures import check_updates, mlm_fixture
    w, trd, dvd, hp, g = mlm_fixture()
    tr = MLMTrainer(w, BERT_TINY, lr=hp["lr"], **NO_DROP)
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
        tr = RescoreBertTrainer(w, BERT_TINY, method="MD_MWED", md_loss_weight=0.3, lr=5e-4, **NO_DROP)
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
    tr = MLMTrainer(w, BERT_TINY, lr=1e-3, **NO_DROP)
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
        tr = MLMTrainer(w, BERT_TINY, lr=1e-3, **NO_DROP)
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


# ---- dropout (BERT train mode, RescoreBert/main.py:83-85, MLM_PLL/main.py:75) ----------------

def test_dropout_keep_bits_statistics():
    """The counter-based keep bits: P(keep) = 1 - p, independent across elements, sites, steps
    and seeds, all ones at p = 0, and the same bits on every call."""
    from asr_rescoring_amd.train import dropout_keep
    n = 1 << 22
    k = dropout_keep(7, 0, 2, 0.1, n).astype(np.float64)
    assert abs(k.mean() - 0.9) < 5 * np.sqrt(0.09 / n)
    assert np.array_equal(k, dropout_keep(7, 0, 2, 0.1, n))
    for other in (dropout_keep(7, 0, 3, 0.1, n), dropout_keep(7, 1, 2, 0.1, n), dropout_keep(8, 0, 2, 0.1, n)):
        agree = (k == other).mean()                  # independent Bernoulli(0.9) pairs: 0.82
        assert abs(agree - 0.82) < 5 * np.sqrt(0.82 * 0.18 / n), agree
    # neighbours within a 64-element run are uncorrelated (no lattice in the counter)
    c = np.corrcoef(k[:-1], k[1:])[0, 1]
    assert abs(c) < 5 / np.sqrt(n)
    assert (dropout_keep(7, 0, 2, 0.0, 1000) == 1).all()
    assert abs(dropout_keep(1, 2, 3, 0.5, n).mean() - 0.5) < 5 * np.sqrt(0.25 / n)


def _keep_fn(tr, seed, step, p_h, p_a):
    from asr_rescoring_amd.train import dropout_keep
    return lambda site, n: dropout_keep(seed, step, site, p_a if site % 3 == 1 else p_h, n)


@pytest.mark.parametrize("method", ["MD", "MD_MWER"])
def test_dropout_gradients_match_oracle_fed_the_same_masks(method):
    """RescoreBert training step at p = 0.1 (hidden and attention): the trainer's masks,
    exported and fed to the torch-autograd oracle, give the same loss, scores and gradients at
    the dropout-free tolerances; the dev pass (update = "loss") is eval mode (no dropout); an
    AdamW step with dropout matches torch.optim.AdamW; and the same seed gives the same step."""
    from asr_rescoring_amd.train import RescoreBertTrainer
    from oracle.train_ref import TorchTrainer, padded_drop
    w = _weights(11)
    nb, seqs, target, am, cer = _batch(70)
    S = BERT_TINY
    tr = RescoreBertTrainer(w, S, method=method, md_loss_weight=0.5, lr=1e-3, dropout_seed=1234)
    ref = TorchTrainer(w, S, lr=1e-3)
    try:
        key = tr.dropout_step()
        loss, sc = tr.step(nb.tokens, nb.hyp_off, nb.utt_off, target, am, cer, update=False)
        assert tr.dropout_step() == key + 1
        drop = padded_drop(_keep_fn(tr, 1234, key, 0.1, 0.1), np.diff(nb.hyp_off), S.hidden, S.heads, S.layers,
                           0.1, 0.1)
        rloss, rsc = ref.step(seqs, target, am, cer, n_best=4, method=method, md_loss_weight=0.5, update=False,
                              drop=drop)
        assert abs(loss - rloss) <= 1e-4 * abs(rloss), (loss, rloss)
        assert np.abs(sc - rsc).max() <= 1e-4 * np.abs(rsc).max()
        gnorm = np.sqrt(sum(float(np.sum(ref.grad(k).astype(np.float64) ** 2)) for k in tr.shapes))
        for k in tr.shapes:
            g, rg = tr.grad(k), ref.grad(k)
            rel = np.linalg.norm(g - rg) / max(np.linalg.norm(rg), 1e-4 * gnorm)
            assert rel < 2e-4, (k, rel)
        # without the masks the oracle disagrees: dropout really was applied
        nl, _ = ref.step(seqs, target, am, cer, n_best=4, method=method, md_loss_weight=0.5, update="loss")
        assert abs(nl - loss) > 1e-3 * abs(nl)
        # dev pass: eval mode, no dropout, the counter does not move
        l_eval, _ = tr.step(nb.tokens, nb.hyp_off, nb.utt_off, target, am, cer, update="loss")
        assert abs(l_eval - nl) <= 1e-4 * abs(nl) and tr.dropout_step() == key + 1
        # one AdamW step with dropout, both sides
        key = tr.dropout_step()
        tr.step(nb.tokens, nb.hyp_off, nb.utt_off, target, am, cer, update=True)
        drop = padded_drop(_keep_fn(tr, 1234, key, 0.1, 0.1), np.diff(nb.hyp_off), S.hidden, S.heads, S.layers,
                           0.1, 0.1)
        ref.step(seqs, target, am, cer, n_best=4, method=method, md_loss_weight=0.5, update=True, drop=drop)
        for k in tr.shapes:
            if k.endswith("attention.self.key.bias"):
                continue        # exactly-zero gradient: AdamW steps on rounding noise (check_updates)
            d, rd = tr.tensor(k) - w[k].reshape(tr.shapes[k]), ref.tensor(k) - w[k].reshape(tr.shapes[k])
            assert np.linalg.norm(d - rd) <= 2e-2 * max(np.linalg.norm(rd), 1e-12), k
    finally:
        tr.close()
    # bitwise reproducible for a seed; another seed draws other masks
    res = {}
    for seed in (1234, 1234, 99):
        t2 = RescoreBertTrainer(w, S, method=method, md_loss_weight=0.5, lr=1e-3, dropout_seed=seed)
        try:
            res.setdefault(seed, []).append(t2.step(nb.tokens, nb.hyp_off, nb.utt_off, target, am, cer,
                                                    update=False)[0])
        finally:
            t2.close()
    assert res[1234][0] == res[1234][1] and res[99][0] != res[1234][0]


def test_mlm_dropout_matches_oracle_fed_the_same_masks():
    """MLM fine-tuning step (padded do_job batch, pads are queries but not keys) at p = 0.1:
    loss and every gradient vs torch autograd fed the trainer's masks."""
    from asr_rescoring_amd.train import MLMTrainer, do_job_rows, pad_rows
    from oracle.train_ref import TorchTrainer, padded_drop
    S = BERT_TINY
    w = make_weights(S, seed=12)
    nb, seqs, *_ = _batch(80, n_utt=2, n_best=3, len_hi=12)
    ids, off, lab = do_job_rows(seqs)
    rows = [ids[off[i]:off[i + 1]].tolist() for i in range(len(off) - 1)]
    labs = [lab[off[i]:off[i + 1]].tolist() for i in range(len(off) - 1)]
    tr = MLMTrainer(w, S, lr=1e-3, dropout_seed=5)
    ref = TorchTrainer(w, S, lr=1e-3, head="mlm")
    try:
        key = tr.dropout_step()
        pid, poff, plab, klen = pad_rows(rows, labs)
        l = tr.step(pid, poff, plab, klen, update=False)
        T = int(poff[1] - poff[0])
        # the trainer's rows are the padded rows (every row T tokens long)
        drop = padded_drop(_keep_fn(tr, 5, key, 0.1, 0.1), [T] * len(rows), S.hidden, S.heads, S.layers, 0.1, 0.1)
        rl = ref.step_mlm(rows, labs, update=False, drop=drop)
        assert abs(l - rl) <= 1e-4 * abs(rl), (l, rl)
        gn = np.sqrt(sum(float(np.sum(ref.model.w[k].grad.numpy().astype(np.float64) ** 2)) for k in tr.shapes))
        for k in tr.shapes:
            g, rg = tr.grad(k), ref.model.w[k].grad.numpy()
            rel = np.linalg.norm(g - rg) / max(np.linalg.norm(rg), 1e-4 * gn)
            assert rel < 2e-4, (k, rel)
    finally:
        tr.close()
