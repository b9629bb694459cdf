"""GPU parity of the BERTScore MBR utility (bertscore.py, k_bertscore.hip) against the
oracle restatement of bert_score (oracle/bertscore_ref.py), including bert_score's batch
padding (a padded position's masked cosine 0 joins the max) at the reference's call pattern
(RMBR/mbr.py pair list, RMBR config batch_size 128) and at small batch sizes where most
pairs are padded.

Tolerance (the default fp16x3 mode: fp32-class encoder, two-part embeddings, split-operand
cosines): recall / P / F within 1e-5 of the fp32 oracle, and the MBR argmax equal for every
utterance and every k.  The opt-in fp16 mode (fp16 embeddings and cosines) is reduced
precision and held to 1e-3 relative (north_star's score tolerance, floored at 0.1)."""
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


TOL32 = 1e-5        # fp16x3 (fp32-class) recall / P / F vs the fp32 oracle, absolute


def _check(scorer, model, nb, which="R"):
    from oracle import bertscore_ref as B
    rmat, rmat0, moff = scorer.recall_matrices(nb.tokens, nb.hyp_off, nb.utt_off)
    got, got0 = rmat.cpu().numpy(), rmat0.cpu().numpy()
    pr = B.pair_recall(model, _utts(nb))
    want = np.concatenate([r.ravel() for r, _ in pr])
    want0 = np.concatenate([r0.ravel() for _, r0 in pr])
    for g, w in ((got, want), (got0, want0)):
        if scorer.precision == "fp16x3":
            assert np.abs(g - w).max() < TOL32, (np.abs(g - w).max(), np.argmax(np.abs(g - w)))
        else:
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
    for prec in ("fp16x3", "fp16"):
        s = BertScorer(w, BERT_TINY, num_layers=2, device=0, max_rows=4096, precision=prec)
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
                assert np.abs(a - b).max() < TOL32
        for which in ("P", "R", "F"):
            for k in (2, 5, 8):
                for bsz in (6, 128):
                    am, sc = BS.mbr_decode(s, nb, k, which, batch_size=bsz)
                    wam, wsc = B.rmbr_mbr_decode(model, utts, k, which, batch_size=bsz)
                    assert np.abs(sc - wsc).max() < k * TOL32, (which, k, bsz)
                    # the MBR pick itself: every utterance, every k (no margin exemption)
                    assert np.array_equal(am, wam), (which, k, bsz)
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
                assert np.abs(sc - wsc).max() < k * TOL32, (k, bsz)
                assert np.array_equal(am, wam), (k, bsz)
        cands = [h for u in utts for h in u]
        refs = [u[-1] for u in utts for _ in u]
        P, R, F = s.score(cands, refs, batch_size=3)
        wp, wr, wf = B.bert_score(model, cands, refs, batch_size=3)
        for a, b in ((P, wp), (R, wr), (F, wf)):
            assert np.abs(a - b).max() < TOL32
    finally:
        s.close()


def test_embed_rows_are_unit_norm():
    from asr_rescoring_amd.bertscore import BertScorer
    from oracle import bertscore_ref as B
    w = make_weights(BERT_TINY, seed=2)
    nb = D.synthetic_nbest(2, 4, seed=1, vocab=BERT_TINY.vocab, len_lo=2, len_hi=20)
    model = B.truncated_model(w, BERT_TINY, 2)
    ref = B.embed_sentences(model, _utts(nb)[0])
    r0 = torch.cat(ref)
    r0 = r0 / r0.norm(dim=1, keepdim=True)
    # fp16x3: fp32-class rows (two-part image); fp16: fp16 rows
    for prec, tol_n, tol_e in (("fp16x3", 1e-6, 2e-6), ("fp16", 2e-3, 5e-3)):
        s = BertScorer(w, BERT_TINY, num_layers=2, device=0, precision=prec)
        try:
            e = s.embed(nb.tokens, nb.hyp_off).float().cpu()
        finally:
            s.close()
        assert torch.allclose(e.norm(dim=1), torch.ones(e.shape[0]), atol=tol_n), prec
        assert (e[:r0.shape[0]] - r0).abs().max() < tol_e, prec


def test_c5_shape_bertscore_mbr_every_utterance_and_k(golden_dir):
    """C5 shape with the BERTScore utility (RMBR/mbr.py:5-28 + RMBR/main.py:15-35, RMBR
    config batch_size 128): bert-base truncated to 8 layers, 3 utterances x N=100 with real
    lengths; the recall matrices within 1e-5 of the fp32 oracle and the MBR argmax equal for
    every utterance and every k in {2, 3, 5, 10, 50, 100} (P, R and F)."""
    import json
    import os
    from asr_rescoring_amd import bertscore as BS
    from oracle import bertscore_ref as B
    lc = json.load(open(os.path.join(golden_dir, "alfred_test_lengths.json")))["length_counts"]
    nb = D.synthetic_nbest(3, 100, seed=33, lengths=np.repeat(np.arange(len(lc)), lc), hard=True)
    w = make_weights(BERT_BASE, seed=3)
    model = B.truncated_model(w, BERT_BASE, 8)
    s = BS.BertScorer(w, BERT_BASE, num_layers=8, device=0, max_rows=65536)
    try:
        _check(s, model, nb)
        rmat, rmat0, moff = s.recall_matrices(nb.tokens, nb.hyp_off, nb.utt_off)
    finally:
        s.close()
    # the oracle's utility matrices from its own recall (per pair, as bert_score pads them)
    utts = _utts(nb)
    for which in ("P", "R", "F"):
        for k in (2, 3, 5, 10, 50, 100):
            util = BS.rmbr_utility(rmat, rmat0, moff, nb.hyp_off, nb.utt_off, k, which, 128)
            am, sc = BS._mbr_on_utility(util, k)
            wam, wsc = B.rmbr_mbr_decode(model, utts, k, which, batch_size=128)
            assert np.abs(sc - wsc).max() < k * TOL32, (which, k)
            assert np.array_equal(am, wam), (which, k)
