"""Host logic of the BERTScore utility (no GPU): the per-pair choice between the plain and the
0-clamped recall matrices that reproduces bert_score's batch padding at the reference's call
pattern (RMBR/mbr.py:5-16 pair list; bert_score bert_cos_score_idf batches), checked against a
loop-by-loop restatement on synthetic matrices whose plain and clamped values differ."""
import numpy as np
import torch

from asr_rescoring_amd import bertscore as BS


def _loop_utility(R, R0, lens, k, bsz, which):
    """The reference's order, one pair at a time: cand i (k-1 copies), refs = the others."""
    pairs = []
    for u, (r, r0, ln) in enumerate(zip(R, R0, lens)):
        for i in range(k):
            for j in list(range(i)) + list(range(i + 1, k)):
                pairs.append((u, i, j, ln[i], ln[j]))
    out = np.zeros((len(R), k, k), np.float32)
    for b0 in range(0, len(pairs), bsz):
        batch = pairs[b0:b0 + bsz]
        cmax = max(p[3] for p in batch)
        rmax = max(p[4] for p in batch)
        for u, i, j, lc, lr in batch:
            rv = R0[u][i, j] if lc < cmax else R[u][i, j]
            pv = R0[u][j, i] if lr < rmax else R[u][j, i]
            if which == "R":
                v = rv
            elif which == "P":
                v = pv
            else:
                with np.errstate(invalid="ignore", divide="ignore"):
                    v = np.float32(2) * pv * rv / (pv + rv)
                v = 0.0 if np.isnan(v) else v
            out[u, i, j] = v
    return out


def test_rmbr_utility_matches_loop_restatement():
    rng = np.random.default_rng(0)
    n_u = [7, 9, 7, 12]
    R = [rng.uniform(-0.5, 1, (n, n)).astype(np.float32) for n in n_u]
    R0 = [np.maximum(r, 0) + rng.uniform(0, 0.1, r.shape).astype(np.float32) for r in R]
    lens = [rng.integers(2, 12, n) for n in n_u]
    uoff = np.concatenate([[0], np.cumsum(n_u)]).astype(np.int32)
    hoff = np.concatenate([[0], np.cumsum(np.concatenate(lens))]).astype(np.int32)
    moff = np.concatenate([[0], np.cumsum([n * n for n in n_u])]).astype(np.int64)
    rmat = torch.from_numpy(np.concatenate([r.ravel() for r in R]))
    rmat0 = torch.from_numpy(np.concatenate([r.ravel() for r in R0]))
    for k in (2, 5, 7):
        for bsz in (1, 4, 13, 128):
            for which in ("R", "P", "F"):
                got = BS.rmbr_utility(rmat, rmat0, moff, hoff, uoff, k, which, bsz).numpy()
                want = _loop_utility(R, R0, lens, k, bsz, which)
                assert np.allclose(got, want, rtol=1e-6, atol=1e-7), (k, bsz, which)


def test_pair_pad_flags():
    lc = np.array([3, 5, 5, 2, 9, 9, 4])
    lr = np.array([4, 4, 6, 6, 1, 2, 3])
    pc, pr = BS.pair_pad_flags(lc, lr, 3)
    assert pc.tolist() == [True, False, False, True, False, False, False]
    assert pr.tolist() == [True, True, False, False, True, True, False]
    tc, tr = BS.pair_pad_flags(torch.from_numpy(lc), torch.from_numpy(lr), 3)
    assert tc.tolist() == pc.tolist() and tr.tolist() == pr.tolist()
