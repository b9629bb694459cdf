"""ORACLE (test infrastructure only) — PyTorch-CPU fp32 restatement of the BERTScore MBR
utility (RMBR/utility_functions.py:9-22 -> ``bert_score.score(cands, refs, lang="zh")``).

``bert_score`` is a third-party dependency that is NOT installed here and is unpinned by the
reference (no requirements file); its published algorithm (bert_score 0.3.x,
``bert_score/score.py`` + ``bert_score/utils.py``) is restated below:

* ``get_model``: the encoder truncated to ``num_layers`` (8 for bert-base-chinese);
  ``bert_encode`` returns that truncated model's last hidden state.
* ``score(idf=False)``: idf weight 1 for every token except [CLS] and [SEP] (0).
* ``bert_cos_score_idf``: unique sentences embedded once; pairs processed in batches of
  ``batch_size`` (library default 64; the reference's RMBR config passes 128), each side padded
  with ``pad_batch_stats`` (embedding pad value 2.0, idf pad 0, mask = real length) — so a
  padded position's masked cosine 0 joins the other side's max.
* ``greedy_cos_idf``: embeddings divided by their L2 norm; ``sim = bmm(hyp, ref^T) * masks``;
  P = sum(max over ref of sim * hyp_idf / sum hyp_idf), R = same over ref; F = 2PR/(P+R);
  P and R set to 0 when a side has only [CLS][SEP]; NaN F set to 0.

The encoder math is ``oracle.bert_ref.TorchBert`` (pinned to the reference via the golden
fixtures); the embedding step is additionally checked against ``transformers.BertModel``
(the class bert_score loads) in tests/test_oracle_bertscore.py.  The greedy matching itself
is **parity unpinned** (no bert_score output is available offline).

Only ``tests/`` and ``bench.py``'s ``cpu_baseline`` leg may import this module.
"""
from __future__ import annotations

import dataclasses
from typing import Dict, List, Sequence, Tuple

import numpy as np
import torch

from .bert_ref import TorchBert
from .rescore_ref import torch_cpu_sum_f32


def truncated_model(weights: Dict[str, np.ndarray], shape, num_layers: int) -> TorchBert:
    keep = {k: v for k, v in weights.items()
            if not k.startswith("bert.encoder.layer.") or int(k.split(".")[3]) < num_layers}
    return TorchBert(keep, dataclasses.replace(shape, layers=num_layers))


def embed_sentences(model: TorchBert, sents: Sequence[Sequence[int]], batch_size: int = 64
                    ) -> List[torch.Tensor]:
    """get_bert_embedding over unique sentences (pad id 0, attention mask = real length)."""
    out: List[torch.Tensor] = [None] * len(sents)
    for b0 in range(0, len(sents), batch_size):
        chunk = list(range(b0, min(len(sents), b0 + batch_size)))
        T = max(len(sents[i]) for i in chunk)
        ids = torch.zeros(len(chunk), T, dtype=torch.long)
        am = torch.zeros(len(chunk), T, dtype=torch.long)
        for r, i in enumerate(chunk):
            ids[r, :len(sents[i])] = torch.as_tensor(np.asarray(sents[i], np.int64))
            am[r, :len(sents[i])] = 1
        with torch.no_grad():
            h = model.encoder(ids, am)
        for r, i in enumerate(chunk):
            out[i] = h[r, :len(sents[i])].clone()
    return out


def _pad_batch_stats(embs: List[torch.Tensor], idfs: List[torch.Tensor]):
    lens = [e.shape[0] for e in embs]
    T = max(lens)
    H = embs[0].shape[1]
    emb = torch.full((len(embs), T, H), 2.0)
    idf = torch.zeros(len(embs), T)
    mask = torch.zeros(len(embs), T, dtype=torch.long)
    for r, (e, w) in enumerate(zip(embs, idfs)):
        emb[r, :e.shape[0]] = e
        idf[r, :e.shape[0]] = w
        mask[r, :e.shape[0]] = 1
    return emb, mask, idf


def greedy_cos_idf(ref_emb, ref_mask, ref_idf, hyp_emb, hyp_mask, hyp_idf):
    ref_emb = ref_emb / torch.norm(ref_emb, dim=-1).unsqueeze(-1)
    hyp_emb = hyp_emb / torch.norm(hyp_emb, dim=-1).unsqueeze(-1)
    sim = torch.bmm(hyp_emb, ref_emb.transpose(1, 2))
    masks = torch.bmm(hyp_mask.unsqueeze(2).float(), ref_mask.unsqueeze(1).float())
    sim = sim * masks
    word_precision = sim.max(dim=2)[0]
    word_recall = sim.max(dim=1)[0]
    hyp_idf = hyp_idf / hyp_idf.sum(dim=1, keepdim=True)
    ref_idf = ref_idf / ref_idf.sum(dim=1, keepdim=True)
    P = (word_precision * hyp_idf).sum(dim=1)
    R = (word_recall * ref_idf).sum(dim=1)
    F = 2 * P * R / (P + R)
    hyp_zero = hyp_mask.sum(dim=1).eq(2)
    ref_zero = ref_mask.sum(dim=1).eq(2)
    P = P.masked_fill(hyp_zero, 0.0).masked_fill(ref_zero, 0.0)
    R = R.masked_fill(hyp_zero, 0.0).masked_fill(ref_zero, 0.0)
    F = F.masked_fill(torch.isnan(F), 0.0)
    return P, R, F


def bert_score(model: TorchBert, cands: Sequence[Sequence[int]], refs: Sequence[Sequence[int]],
               cls_id: int = 101, sep_id: int = 102, batch_size: int = 64
               ) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """bert_score.score(cands, refs, idf=False) on token-id sentences ([CLS] w.. [SEP])."""
    uniq = sorted({tuple(s) for s in list(refs) + list(cands)}, key=len, reverse=True)
    embs = embed_sentences(model, [list(s) for s in uniq], batch_size)
    stats = {}
    for s, e in zip(uniq, embs):
        w = torch.tensor([0.0 if t in (cls_id, sep_id) else 1.0 for t in s])
        stats[s] = (e, w)
    P, R, F = [], [], []
    for b0 in range(0, len(refs), batch_size):
        rs = [stats[tuple(s)] for s in refs[b0:b0 + batch_size]]
        hs = [stats[tuple(s)] for s in cands[b0:b0 + batch_size]]
        re, rm, ri = _pad_batch_stats([e for e, _ in rs], [w for _, w in rs])
        he, hm, hi = _pad_batch_stats([e for e, _ in hs], [w for _, w in hs])
        p, r, f = greedy_cos_idf(re, rm, ri, he, hm, hi)
        P.append(p), R.append(r), F.append(f)
    cat = lambda x: torch.cat(x).numpy().astype(np.float32)
    return cat(P), cat(R), cat(F)


def utility_matrices(model: TorchBert, utts: List[List[Sequence[int]]], which: str = "R",
                     **kw) -> List[np.ndarray]:
    """sim[i, j] = bert_score(cand = hyp_i, ref = hyp_j)[which] for every ordered pair."""
    cands, refs, where = [], [], []
    for u, hyps in enumerate(utts):
        for i in range(len(hyps)):
            for j in range(len(hyps)):
                cands.append(list(hyps[i])), refs.append(list(hyps[j])), where.append((u, i, j))
    P, R, F = bert_score(model, cands, refs, **kw)
    val = {"P": P, "R": R, "F": F}[which]
    mats = [np.zeros((len(h), len(h)), np.float32) for h in utts]
    for (u, i, j), v in zip(where, val):
        mats[u][i, j] = v
    return mats


def pair_recall(model: TorchBert, utts: List[List[Sequence[int]]]) -> List[Tuple[np.ndarray, np.ndarray]]:
    """Per utterance, for every ordered pair (cand i, ref j) of its hypotheses without any batch
    padding: R[i, j] = mean over ref j's tokens except [CLS]/[SEP] of the max cosine over all of
    cand i's tokens, and R0[i, j] with each max clamped at 0 (the value a padded cand gets in
    bert_score's masked max); 0 when either side is empty ([CLS][SEP])."""
    out = []
    for hyps in utts:
        embs = embed_sentences(model, [list(h) for h in hyps])
        embs = [e / torch.norm(e, dim=-1, keepdim=True) for e in embs]
        n = len(hyps)
        R, R0 = np.zeros((n, n), np.float32), np.zeros((n, n), np.float32)
        for i in range(n):
            for j in range(n):
                if len(hyps[i]) <= 2 or len(hyps[j]) <= 2:
                    continue
                m = (embs[i] @ embs[j].t()).max(dim=0)[0][1:-1]
                R[i, j] = float(m.mean())
                R0[i, j] = float(m.clamp_min(0.0).mean())
        out.append((R, R0))
    return out


def rmbr_mbr_decode(model: TorchBert, utts: List[List[Sequence[int]]], k: int, which: str = "R",
                    batch_size: int = 128) -> Tuple[np.ndarray, np.ndarray]:
    """RMBR/mbr.py:5-28 with BertScoreFunction (RMBR/utility_functions.py:9-22): the pair list
    (cand = hyp i repeated k-1 times, refs = the other hyps of the top k), one bert_score call
    over it in batches of ``batch_size`` (RMBR config: 128), scores reshaped to [U, k, k-1],
    float32 torch-CPU sum, first max."""
    cands, refs = [], []
    for hyps in utts:
        for i in range(k):
            cands += [list(hyps[i])] * (k - 1)
            refs += [list(h) for h in hyps[:i] + hyps[i + 1:k]]
    P, R, F = bert_score(model, cands, refs, batch_size=batch_size)
    val = {"P": P, "R": R, "F": F}[which].reshape(len(utts), k, k - 1)
    scores = np.zeros((len(utts), k), np.float32)
    for u in range(len(utts)):
        for i in range(k):
            scores[u, i] = torch_cpu_sum_f32(val[u, i])
    return np.argmax(scores, axis=-1), scores


def mbr_decode(k: int, mats: List[np.ndarray]) -> Tuple[np.ndarray, np.ndarray]:
    """RMBR/mbr.py:5-28 with a precomputed utility: sims j = 0..i-1, i+1..k-1 of cand i,
    float32 torch-CPU sum, first max."""
    scores = np.zeros((len(mats), k), np.float32)
    for u, m in enumerate(mats):
        for i in range(k):
            sims = [m[i, j] for j in list(range(0, i)) + list(range(i + 1, k))]
            scores[u, i] = torch_cpu_sum_f32(np.asarray(sims, np.float32))
    return np.argmax(scores, axis=-1), scores
