"""GPU parity of the BERTScore MBR utility (bertscore.py, k_bertscore.hip) against the
oracle restatement of bert_score (oracle/bertscore_ref.py), including bert_score's batch
padding (a padded position's masked cosine 0 joins the max) at the reference's call pattern
(RMBR/mbr.py pair list, RMBR config batch_size 128) and at small batch sizes where most
pairs are padded.

Tolerance: R/P/F within 1e-3 relative of the fp32 oracle (north_star's score tolerance);
MBR argmax equal wherever the oracle's best and second-best sums differ by more than the
accumulated tolerance."""
import numpy as np
import pytest
import torch

from asr_rescoring_amd import data as D
from asr_rescoring_amd.weights import BERT_BASE, BERT_TINY, make_weights

pytestmark = pytest.mark.gpu

REL = 1e-3


def _utts(nb):
    return [[nb.tokens[nb.hyp_off[h]:nb.hyp_off[h + 1]].tolist() for h in range(nb.utt_off[u], nb.utt_off[u + 1])]
            for u in range(nb.n_utt)]


def _check(scorer, model, nb, which="R"):
    from oracle import bertscore_ref as B
    rmat, rmat0, moff = scorer.recall_matrices(nb.tokens, nb.hyp_off, nb.utt_off)
    got, got0 = rmat.cpu().numpy(), rmat0.cpu().numpy()
    pr = B.pair_recall(model, _utts(nb))
    want = np.concatenate([r.ravel() for r, _ in pr])
    want0 = np.concatenate([r0.ravel() for _, r0 in pr])
    for g, w in ((got, want), (got0, want0)):
        # relative, floored at 0.1: recalls near 0 (isotropic embeddings) carry the fp16
        # embedding rounding as an absolute error
        err = np.abs(g - w) / np.maximum(np.abs(w), 0.1)
        assert err.max() < REL, (err.max(), np.argmax(err))
    return [r for r, _ in pr]


@pytest.mark.parametrize("shape,layers,precision", [(BERT_TINY, 2, "fp16"), (BERT_BASE, 8, "fp16"),
                                                     (BERT_BASE, 8, "fp16x3")])
def test_recall_matrix_vs_oracle(shape, layers, precision):
    from asr_rescoring_amd.bertscore import BertScorer
    from oracle import bertscore_ref as B
    w = make_weights(shape, seed=3)
    nb = D.synthetic_nbest(3, 7, seed=4, vocab=shape.vocab, len_lo=1, len_hi=30)
    s = BertScorer(w, shape, num_layers=layers, device=0, max_rows=4096, precision=precision)
    try:
        _check(s, B.truncated_model(w, shape, layers), nb)
    finally:
        s.close()


def test_long_hypotheses_and_many_candidates():
    """T > 64 (a ref walked in several 64-column sub-tiles) and n_u > 128 (candidate groups),
    plus empty hypotheses ([CLS][SEP]: P = R = 0)."""
    from asr_rescoring_amd.bertscore import BertScorer
    from oracle import bertscore_ref as B
    w = make_weights(BERT_TINY, seed=5)
    rng = np.random.default_rng(6)
    utt0 = [rng.integers(106, BERT_TINY.vocab, size=L).tolist() for L in (70, 150, 3, 0, 65, 1)]
    utt1 = [rng.integers(106, BERT_TINY.vocab, size=int(rng.integers(0, 6))).tolist() for _ in range(140)]
    nb = D.from_lists([utt0, utt1])
    s = BertScorer(w, BERT_TINY, num_layers=2, device=0, max_rows=4096)
    try:
        mats = _check(s, B.truncated_model(w, BERT_TINY, 2), nb)
    finally:
        s.close()
    assert mats[0][3].max() == 0.0 and mats[0][:, 3].max() == 0.0


def test_score_pairs_and_mbr():
    from asr_rescoring_amd import bertscore as BS
    from oracle import bertscore_ref as B
    w = make_weights(BERT_TINY, seed=8)
    model = B.truncated_model(w, BERT_TINY, 2)
    nb = D.synthetic_nbest(6, 8, seed=9, vocab=BERT_TINY.vocab, len_lo=1, len_hi=24)
    s = BS.BertScorer(w, BERT_TINY, num_layers=2, device=0, max_rows=4096)
    try:
        utts = _utts(nb)
        cands = [h for u in utts for h in u]
        refs = [u[0] for u in utts for _ in u]
        for bsz in (4, 64):
            P, R, F = s.score(cands, refs, batch_size=bsz)
            wp, wr, wf = B.bert_score(model, cands, refs, batch_size=bsz)
            for a, b in ((P, wp), (R, wr), (F, wf)):
                assert (np.abs(a - b) / np.maximum(np.abs(b), 1e-6)).max() < REL
        for which in ("P", "R", "F"):
            for k in (2, 5, 8):
                for bsz in (6, 128):
                    am, sc = BS.mbr_decode(s, nb, k, which, batch_size=bsz)
                    wam, wsc = B.rmbr_mbr_decode(model, utts, k, which, batch_size=bsz)
                    assert np.allclose(sc, wsc, rtol=REL, atol=1e-5), (which, k, bsz)
                    top2 = np.sort(wsc, axis=1)[:, -2:]
                    clear = (top2[:, 1] - top2[:, 0]) > 2e-3 * np.abs(top2[:, 1])
                    assert (am[clear] == wam[clear]).all()
        cer, best_k, _ = BS.find_best_length(s, nb, 8)
        assert 0.0 <= cer <= 1.0 and 2 <= best_k <= 8
    finally:
        s.close()


def _isotropic_weights(seed):
    """Tiny BERT whose layers pass the embeddings through (zero attention / FFN output
    projections, identity LayerNorms) and whose position / type embeddings are zero: token
    vectors are LN(random word embedding), so cosines between different tokens scatter around
    0 and short hypotheses leave ref tokens with a negative best cosine."""
    w = make_weights(BERT_TINY, seed=seed)
    for k in list(w):
        if "position_embeddings" in k or "token_type_embeddings" in k or "attention.output.dense" in k \
                or (".output.dense." in k and "attention" not in k):
            w[k] = np.zeros_like(w[k])
        elif "LayerNorm.weight" in k:
            w[k] = np.ones_like(w[k])
        elif "LayerNorm.bias" in k:
            w[k] = np.zeros_like(w[k])
    return w


def test_batch_padding_changes_scores_where_best_cosine_is_negative():
    """Where a ref token's best cosine is negative, a padded cand scores max(., 0) there
    (bert_score's masked pad positions): the clamped matrix differs from the plain one, and
    scores at the reference's call pattern follow the oracle's literal batch loop."""
    from asr_rescoring_amd import bertscore as BS
    from oracle import bertscore_ref as B
    w = _isotropic_weights(12)
    model = B.truncated_model(w, BERT_TINY, 2)
    nb = D.synthetic_nbest(8, 6, seed=13, vocab=BERT_TINY.vocab, len_lo=1, len_hi=4)
    s = BS.BertScorer(w, BERT_TINY, num_layers=2, device=0, max_rows=4096)
    try:
        _check(s, model, nb)
        rmat, rmat0, _ = s.recall_matrices(nb.tokens, nb.hyp_off, nb.utt_off)
        assert bool((rmat0 != rmat).any())
        utts = _utts(nb)
        for k in (3, 6):
            for bsz in (5, 128):
                am, sc = BS.mbr_decode(s, nb, k, "R", batch_size=bsz)
                wam, wsc = B.rmbr_mbr_decode(model, utts, k, "R", batch_size=bsz)
                assert np.allclose(sc, wsc, rtol=REL, atol=1e-5), (k, bsz)
        cands = [h for u in utts for h in u]
        refs = [u[-1] for u in utts for _ in u]
        P, R, F = s.score(cands, refs, batch_size=3)
        wp, wr, wf = B.bert_score(model, cands, refs, batch_size=3)
        for a, b in ((P, wp), (R, wr), (F, wf)):
            assert np.allclose(a, b, rtol=REL, atol=1e-5)
    finally:
        s.close()


def test_embed_rows_are_unit_norm():
    from asr_rescoring_amd.bertscore import BertScorer
    from oracle import bertscore_ref as B
    w = make_weights(BERT_TINY, seed=2)
    nb = D.synthetic_nbest(2, 4, seed=1, vocab=BERT_TINY.vocab, len_lo=2, len_hi=20)
    s = BertScorer(w, BERT_TINY, num_layers=2, device=0)
    try:
        e = s.embed(nb.tokens, nb.hyp_off).float().cpu()
    finally:
        s.close()
    assert torch.allclose(e.norm(dim=1), torch.ones(e.shape[0]), atol=2e-3)
    model = B.truncated_model(w, BERT_TINY, 2)
    ref = B.embed_sentences(model, _utts(nb)[0])
    r0 = torch.cat(ref)
    r0 = r0 / r0.norm(dim=1, keepdim=True)
    assert (e[:r0.shape[0]] - r0).abs().max() < 5e-3
