"""The oracle (CPU restatement) pinned against the golden vectors the reference produced.

Fixtures come from tests/golden/make_golden.py, which imported and ran the reference code
(MLM_PLL/main.py run_one_epoch, RescoreBert/model.py, rescore.py, RMBR/mbr.py) on the same
seeded weights/inputs.  These tests need no GPU.
"""
import json
import os

import numpy as np
import pytest
import torch

from asr_rescoring_amd import data as D
from asr_rescoring_amd.weights import BERT_BASE, BERT_TINY, make_weights, weights_digest
from oracle import bert_ref as B
from oracle import rescore_ref as R


def _load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name), allow_pickle=False)


@pytest.fixture(scope="module")
def tiny():
    return make_weights(BERT_TINY, seed=7, with_cls_linear=True, with_pooler=True)


def test_weights_match_fixture_digest(golden_dir, tiny):
    g = _load(golden_dir, "pll_tiny.npz")
    assert weights_digest(tiny) == str(g["digest"])


def test_weights_base_digest(golden_dir):
    g = _load(golden_dir, "pll_base.npz")
    w = make_weights(BERT_BASE, seed=1234, with_cls_linear=True, with_pooler=True)
    assert weights_digest(w) == str(g["digest"])


def test_oracle_pll_tiny(golden_dir, tiny):
    g = _load(golden_dir, "pll_tiny.npz")
    m = B.TorchBert(tiny, BERT_TINY)
    rows, pll = B.pll_reference_pattern(m, g["tokens"], g["hyp_off"], batch_size=32, full_head=True)
    assert np.allclose(rows, g["row_lp"], rtol=2e-5, atol=1e-5)
    assert np.allclose(pll, g["pll"], rtol=2e-6)
    rows2, pll2 = B.pll_reference_pattern(m, g["tokens"], g["hyp_off"], batch_size=7, full_head=False)
    assert np.allclose(pll2, g["pll"], rtol=2e-6)


def test_oracle_cls_tiny(golden_dir, tiny):
    g = _load(golden_dir, "pll_tiny.npz")
    got = B.cls_reference_pattern(B.TorchBert(tiny, BERT_TINY), g["tokens"], g["hyp_off"], with_pooler=True)
    assert np.allclose(got, g["cls"], rtol=1e-5, atol=1e-6)


def test_oracle_pll_base(golden_dir):
    """BERT-base, the F1 fixture (195 masked rows through the reference run_one_epoch)."""
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    g = _load(golden_dir, "pll_base.npz")
    w = make_weights(BERT_BASE, seed=1234)
    m = B.TorchBert(w, BERT_BASE)
    rows, pll = B.pll_reference_pattern(m, g["tokens"], g["hyp_off"], batch_size=32, full_head=False)
    assert np.allclose(rows, g["row_lp"], rtol=2e-5, atol=1e-5)
    assert np.allclose(pll, g["pll"], rtol=2e-6)


def test_oracle_cls_base(golden_dir):
    g = _load(golden_dir, "cls_base.npz")
    w = make_weights(BERT_BASE, seed=1234, with_cls_linear=True, with_pooler=True)
    got = B.cls_reference_pattern(B.TorchBert(w, BERT_BASE), g["tokens"], g["hyp_off"])
    assert np.allclose(got, g["cls"], rtol=1e-5, atol=1e-5)


def test_levenshtein_known_answers():
    # espnet_data/preprocess/align.py:12-18 docstring examples (alignment with 1 and 2 edits)
    assert R.levenshtein_py(["how", "are", "you"], ["how", "are", "you", "doing"]) == 1
    assert R.levenshtein_py(list("你好嗎"), list("你好不好")) == 2
    rng = np.random.default_rng(0)
    for _ in range(300):
        a = rng.integers(0, 5, size=rng.integers(0, 30)).tolist()
        b = rng.integers(0, 5, size=rng.integers(0, 30)).tolist()
        assert R.levenshtein(a, b) == R.levenshtein_py(a, b)
    assert R.levenshtein([], [1, 2, 3]) == 3 and R.levenshtein([4], []) == 1


def test_cer_value_domain_matches_reference_data():
    """hyps_cer.json values are exactly edits/len(ref): corpus CER of one pair."""
    c = R.corpus_cer([[1, 2, 3, 4]], [[1, 9, 3]])
    assert c == 2 / 4
    with pytest.raises(ValueError):
        R.corpus_cer([[]], [[1]])


def test_cer_vs_jiwer_recorded_outputs(golden_dir):
    """jiwer pinned: the reference holds jiwer.cer's outputs for 7176 (ref, pred)
    pairs (Nbest_Align/cer.json; tests/golden/make_jiwer_fixture.py keeps the 1734 with a
    non-zero CER and 200 zero ones).  The restatement (edits of ``strip()``-ed code points /
    ref length, as Python float64) reproduces every recorded value bit for bit, and the corpus
    form (Σ edits / Σ ref chars) the same sum."""
    pairs = json.load(open(os.path.join(golden_dir, "jiwer_cer_pairs.json"), encoding="utf-8"))["pairs"]
    assert len(pairs) == 1934
    refs, hyps = [], []
    for ref, pred, cer in pairs:
        r, h = [ord(c) for c in ref.strip()], [ord(c) for c in pred.strip()]
        assert R.levenshtein(r, h) / len(r) == cer, (ref, pred, cer)
        refs.append(r)
        hyps.append(h)
    edits = sum(round(cer * len(ref.strip())) for ref, _, cer in pairs)
    assert R.corpus_cer(refs, hyps) == edits / sum(len(r) for r in refs)


@pytest.mark.parametrize("n", list(range(1, 100)))
def test_torch_sum_order(n):
    x = torch.rand(64, n) * 0.3 + 0.7
    ref = x.sum(-1).numpy()
    got = np.array([R.torch_cpu_sum_f32(row) for row in x.numpy()])
    assert np.array_equal(ref, got)


def test_rescore_oracle_vs_c1_fixture(golden_dir):
    g = json.load(open(os.path.join(golden_dir, "c1_plumbing.json"), encoding="utf-8"))
    uids = g["utt_ids"]
    am = np.array([list(g["hyps_score"][u].values()) for u in uids])
    lm = np.array([list(g["lm"][u].values()) for u in uids])
    hyps = [[[ord(c) for c in t] for t in g["hyps_text"][u].values()] for u in uids]
    refs = [[ord(c) for c in g["ref_text"][u]] for u in uids]
    best_w, best_cer, args = R.find_best_weight(am, lm, hyps, refs, n_best=10)
    assert np.array_equal(args, np.array(g["argmax_per_weight"]))
    assert best_w == g["best_weight"] and best_cer == g["best_cer"]


def test_mbr_oracle_vs_fixture(golden_dir):
    g = _load(golden_dir, "rmbr.npz")
    tok, off, uoff = g["tokens"], g["hyp_off"], g["utt_off"]
    hyps = [[tok[off[h] + 1:off[h + 1] - 1].tolist() for h in range(uoff[u], uoff[u + 1])]
            for u in range(len(uoff) - 1)]
    for k in range(2, 13):
        idx, sc = R.mbr_decode(k, hyps)
        assert np.array_equal(idx, g[f"argmax_k{k}"])
        assert np.array_equal(sc, g[f"scores_k{k}"])


def test_fusion_modes_formula():
    am = np.array([[-1.0, -2.0], [-3.0, -0.5]])
    lm = np.array([[-10.0, -5.0], [-7.0, -9.0]])
    ln = np.array([[2, 3], [4, 1]])
    w = 0.3
    assert np.array_equal(R.fuse(w, ln, am, lm, "norm"), (1 - w) * am / ln + w * lm / ln)
    assert np.array_equal(R.fuse(w, ln, am, lm, "legacy"), (1 - w) * am + w * lm)
    assert np.array_equal(R.fuse(w, ln, am, lm, "am_norm"), (1 - w) * am / ln + w * lm)
    assert len(R.weight_grid("norm")) == 101 and len(R.weight_grid("legacy")) == 100


def test_data_synthetic_and_json(tmp_path):
    a = D.synthetic_nbest(5, 4, seed=2)
    b = D.synthetic_nbest(5, 4, seed=2)
    assert np.array_equal(a.tokens, b.tokens) and np.array_equal(a.am, b.am)
    assert (np.diff(a.am.reshape(5, 4), axis=1) <= 0).all()          # sorted descending
    lens = a.hyp_len()
    assert lens.min() >= 24 - 3 and lens.max() <= 40 + 3
    sub = a.subset([1, 3])
    assert sub.n_utt == 2 and np.array_equal(sub.hyp_words(0), a.hyp_words(a.utt_off[1]))
    js = D.scores_to_json_dict(a, np.arange(a.n_hyp, dtype=float))
    p = tmp_path / "x.json"
    D.json_saving(str(p), js)
    raw = p.read_text(encoding="utf8")
    assert raw == json.dumps(js, ensure_ascii=False, indent=4)      # util/saving.py:14-16
    assert list(js["utt_0"]) == ["hyp_1", "hyp_2", "hyp_3", "hyp_4"]
    assert B.forward_flops(34, BERT_BASE) == pytest.approx(5.459e9, rel=1e-3)


# ---- training (F6 / F7: the reference's own training loops, tests/golden/make_golden_train.py)
@pytest.mark.parametrize("method", ["MD", "MD_MWER", "MD_MWED"])
def test_oracle_rescorebert_training_vs_reference(method):
    """oracle.train_ref restates RescoreBert/main.py:82-229: two epochs (AdamW per epoch),
    epoch / dev losses, dev scores and every parameter update equal the reference's run."""
    from oracle.train_ref import TorchTrainer, train_rescorebert
    from train_fixtures import check_updates, rb_fixture
    w, tr_d, dv_d, hp, g = rb_fixture(method)
    tr = TorchTrainer(w, BERT_TINY, lr=hp["lr"])
    before = {k: tr.tensor(k).copy() for k in tr.model.w}
    tl, dl = train_rescorebert(tr, tr_d, dv_d, 2, hp["batch_size"], hp["n_best"], method, hp["md_loss_weight"])
    np.testing.assert_allclose(tl, g["train_loss"], rtol=1e-4)
    np.testing.assert_allclose(dl, g["dev_loss"], rtol=1e-4)
    with torch.no_grad():
        sc = tr.scores(dv_d["seqs"]).numpy()
    np.testing.assert_allclose(sc, g["dev_scores"], rtol=1e-4, atol=1e-5)
    check_updates(g, before, {k: tr.tensor(k) for k in tr.model.w})


def test_oracle_mlm_training_vs_reference():
    """oracle.train_ref restates MLM_PLL/main.py:28-161: padded batches with [PAD] labels in
    the CE mean, two epochs, dev loss, parameter updates."""
    from oracle.train_ref import TorchTrainer, train_mlm
    from train_fixtures import check_updates, mlm_fixture
    w, tr_d, dv_d, hp, g = mlm_fixture()
    tr = TorchTrainer(w, BERT_TINY, lr=hp["lr"], head="mlm")
    before = {k: tr.tensor(k).copy() for k in tr.model.w}
    tl, dl = train_mlm(tr, tr_d, dv_d, 2, hp["batch_size"])
    np.testing.assert_allclose(tl, g["train_loss"], rtol=1e-4)
    np.testing.assert_allclose(dl, g["dev_loss"], rtol=1e-4)
    check_updates(g, before, {k: tr.tensor(k) for k in tr.model.w})


def test_alignment_oracle_known_answers():
    """oracle.align_ref vs the reference's docstring examples (espnet_data/preprocess/align.py:12-18)."""
    from oracle.align_ref import levenshtein_distance_alignment as al
    assert al(["how", "are", "you"], ["how", "are", "you", "doing"]) == \
        [["how", "are", "you", "*"], ["how", "are", "you", "doing"], ["U", "U", "U", "D"]]
    assert al(list("你好嗎"), list("你好不好")) == [["你", "好", "*", "嗎"], ["你", "好", "不", "好"], ["U", "U", "D", "S"]]
    assert al([], []) == [[], [], []]
