"""BERTScore MBR utility on the GPU.

The reference's ``BertScoreFunction`` (RMBR/utility_functions.py:9-22) calls
``bert_score.score(cands, refs, lang="zh")``: bert-base-chinese truncated to its first 8
encoder layers, ``idf=False``, no baseline rescaling.  ``bert_score`` is not installed (and
the model is fetched by name), so this module implements the library's published algorithm
on the HIP path:

* ``BertScorer.embed`` — ``get_bert_embedding`` / ``bert_encode``: the last hidden state of
  the truncated encoder for every token, L2-normalised as ``greedy_cos_idf`` does first
  (``rs_token_embed``).  Default precision fp16x3: the encoder's GEMMs, the embeddings (a
  two-part fp16 image, ~22 bits) and the cosines (three fp16 MFMA products) are fp32-class,
  as bert_score computes in fp32.
* ``BertScorer.recall_matrix`` — ``greedy_cos_idf`` for every ordered pair (cand i, ref j)
  of each utterance's hypotheses in one fused MFMA kernel (``rs_bertscore_recall``):
  R(i|j), with P(i|j) = R(j|i) and F = 2PR / (P + R).
* ``BertScorer.score(cands, refs)`` — ``bert_score.score``'s (P, R, F) for aligned lists.
* ``mbr_decode`` / ``find_best_length`` — RMBR/mbr.py:5-28 and RMBR/main.py:15-35 with this
  utility (``rs_mbr_scores_bs``; same float32 summation order and first-max argmax as the
  CER utility in ``rerank``).

Batch padding, as bert_score has it: ``bert_cos_score_idf`` processes the pair list in
batches of ``batch_size`` (bert_score's default 64; the reference's RMBR config passes 128),
pads each side to the longest sentence of its batch and multiplies the cosines by the pad
masks, so when a pair's cand is shorter than the longest cand of its batch the padded
positions offer a cosine of 0 to every ref token's max (and the same for P with the ref
side).  The kernel returns both the plain and the 0-clamped matrices (``rs_bertscore_recall``
``d_rmat`` / ``d_rmat0``), and ``score`` / ``mbr_decode`` / ``find_best_length`` pick one per
pair from the batch layout the reference's call produces (``pair_pad_flags``).
"""
from __future__ import annotations

import dataclasses
from typing import Dict, Sequence, Tuple

import numpy as np
import torch

from . import _lib
from .data import NBest
from .rerank import corpus_edits, ref_edits, _dev
from .scorer import BertEngine
from .weights import BertShape, BERT_BASE

WHICH = {"P": 0, "R": 1, "F": 2}
BERT_SCORE_LAYERS = 8          # bert_score model2layers["bert-base-chinese"]


def truncate_weights(weights: Dict[str, np.ndarray], num_layers: int) -> Dict[str, np.ndarray]:
    """bert_score ``get_model``: keep the embeddings and encoder layers < num_layers.
    Accepts ``BertModel`` keys (``embeddings.*``) or ``bert.*``-prefixed ones."""
    out = {}
    for k, v in weights.items():
        key = k if k.startswith("bert.") else "bert." + k
        if not (key.startswith("bert.embeddings.") or key.startswith("bert.encoder.layer.")):
            continue
        if key.startswith("bert.encoder.layer."):
            if int(key.split(".")[3]) >= num_layers:
                continue
        out[key] = v
    return out


class BertScorer(BertEngine):
    """Encoder-only engine for the BERTScore utility (model truncated to ``num_layers``)."""

    def __init__(self, weights, shape: BertShape = BERT_BASE, num_layers: int = BERT_SCORE_LAYERS,
                 device=0, max_rows: int = 65536, precision: str = "fp16x3"):
        # fp16x3 (default): fp32-class encoder, two-part embeddings and split-operand cosines,
        # as bert_score's fp32 model and matmul; "fp16" is the opt-in reduced-precision mode
        num_layers = min(num_layers, shape.layers)
        sh = dataclasses.replace(shape, layers=num_layers)
        super().__init__(truncate_weights(weights, num_layers), sh, _lib.RS_HEAD_EMB, device, max_rows,
                         precision)

    def embed(self, tokens, hyp_off) -> torch.Tensor:
        """[sum T, H]: L2-normalised last hidden state of every token — float32 (hi + lo/64 of
        the two-part image) in the fp16x3 mode, fp16 in the fp16 mode."""
        off = np.ascontiguousarray(hyp_off, np.int32)
        d_tok = self._dev_tokens(tokens)
        H, two = self.shape.hidden, self.precision == "fp16x3"
        out = torch.empty(int(off[-1]) if len(off) else 0, H * (2 if two else 1), dtype=torch.float16,
                          device=self.device)
        _lib.check(self.lib.rs_token_embed(self.handle, _lib.ptr(d_tok), off.ctypes.data, len(off) - 1,
                                           _lib.ptr(out), _lib.stream_ptr(self.device)))
        if two:
            return out[:, :H].float() + out[:, H:].float() * (1.0 / 64.0)
        return out

    def recall_matrices(self, tokens, hyp_off, utt_off, clamped: bool = True):
        """Concatenated n_u x n_u float32 blocks R[i, j] = R(cand i | ref j), the same with every
        token maximum clamped at 0 (None unless ``clamped``), and the block offsets."""
        hoff = np.ascontiguousarray(hyp_off, np.int32)
        uoff = np.ascontiguousarray(utt_off, np.int32)
        n_u = np.diff(uoff).astype(np.int64)
        moff = np.zeros(len(uoff), np.int64)
        moff[1:] = np.cumsum(n_u * n_u)
        d_tok = self._dev_tokens(tokens)
        rmat = torch.empty(int(moff[-1]), dtype=torch.float32, device=self.device)
        rmat0 = torch.empty_like(rmat) if clamped else None
        _lib.check(self.lib.rs_bertscore_recall(self.handle, _lib.ptr(d_tok), hoff.ctypes.data, uoff.ctypes.data,
                                                len(uoff) - 1, _lib.ptr(rmat), _lib.ptr(rmat0) if clamped else None,
                                                _lib.stream_ptr(self.device)))
        return rmat, rmat0, moff

    def recall_matrix(self, tokens, hyp_off, utt_off) -> Tuple[torch.Tensor, np.ndarray]:
        """Concatenated n_u x n_u float32 blocks R[i, j] = R(cand i | ref j), and their offsets
        (maxima over real tokens only: no batch padding)."""
        rmat, _, moff = self.recall_matrices(tokens, hyp_off, utt_off, clamped=False)
        return rmat, moff

    def score(self, cands: Sequence[Sequence[int]], refs: Sequence[Sequence[int]], batch_size: int = 64
              ) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """``bert_score.score(cands, refs, batch_size=batch_size)`` on token ids ([CLS] w.. [SEP]
        each): (P, R, F), with the batch padding of ``bert_cos_score_idf``."""
        if len(cands) != len(refs):
            raise ValueError("cands and refs differ in length")
        if not cands:
            z = np.zeros(0, np.float32)
            return z, z, z
        seqs = [s for pair in zip(cands, refs) for s in pair]
        hoff = np.zeros(len(seqs) + 1, np.int32)
        hoff[1:] = np.cumsum([len(s) for s in seqs])
        toks = np.concatenate([np.asarray(s, np.int32) for s in seqs])
        uoff = np.arange(0, len(seqs) + 1, 2, dtype=np.int32)
        rmat, rmat0, _ = self.recall_matrices(toks, hoff, uoff)
        r, r0 = rmat.view(-1, 2, 2).cpu().numpy(), rmat0.view(-1, 2, 2).cpu().numpy()
        pad_c, pad_r = pair_pad_flags(np.array([len(c) for c in cands]), np.array([len(x) for x in refs]), batch_size)
        R = np.where(pad_c, r0[:, 0, 1], r[:, 0, 1]).astype(np.float32)    # (cand 0 | ref 1)
        P = np.where(pad_r, r0[:, 1, 0], r[:, 1, 0]).astype(np.float32)    # its transpose
        with np.errstate(invalid="ignore", divide="ignore"):
            F = (np.float32(2) * P * R / (P + R)).astype(np.float32)
        F[np.isnan(F)] = 0.0
        return P, R, F


def pair_pad_flags(len_cand, len_ref, batch_size: int):
    """Per pair of a bert_score call (pairs in list order, ``batch_size`` per batch): is the
    cand / the ref shorter than the longest cand / ref of its batch (so padded positions,
    masked to cosine 0, join the max).  numpy or torch 1-D integer arrays in, bool out."""
    out = []
    for ln in (len_cand, len_ref):
        n = ln.shape[0]
        nb = -(-n // batch_size)
        if isinstance(ln, torch.Tensor):
            padded = torch.zeros(nb * batch_size, dtype=ln.dtype, device=ln.device)
            padded[:n] = ln
            mx = padded.view(nb, batch_size).amax(dim=1).repeat_interleave(batch_size)[:n]
        else:
            padded = np.zeros(nb * batch_size, ln.dtype)
            padded[:n] = ln
            mx = np.repeat(padded.reshape(nb, batch_size).max(axis=1), batch_size)[:n]
        out.append(ln < mx)
    return out[0], out[1]


def rmbr_utility(rmat: torch.Tensor, rmat0: torch.Tensor, moff: np.ndarray, hyp_off, utt_off, k: int,
                 which: str = "R", batch_size: int = 128) -> torch.Tensor:
    """The utility values the reference's mbr_decode (RMBR/mbr.py:5-28) gets from
    ``BertScoreFunction.score(cands, refs)`` for top-k: its pair list (utterance, cand i < k,
    ref j < k, j != i, in that order) scored by bert_score in batches of ``batch_size``,
    returned as [U, k, k] float32 blocks (diagonal 0) for ``rs_mbr_scores_bs``."""
    dev = rmat.device
    uoff = np.ascontiguousarray(utt_off, np.int64)
    U = len(uoff) - 1
    n_u = torch.from_numpy(np.diff(uoff)).to(dev)
    lens = torch.from_numpy(np.diff(np.asarray(hyp_off, np.int64))).to(dev)
    ii = torch.arange(k, device=dev)[:, None].expand(k, k - 1)
    jj = torch.arange(k - 1, device=dev)[None, :].expand(k, k - 1)
    jj = jj + (jj >= ii).long()                                  # refs: hyps[:i] + hyps[i+1:k]
    base = torch.from_numpy(uoff[:-1]).to(dev)[:, None, None]
    mo = torch.from_numpy(np.asarray(moff[:-1], np.int64)).to(dev)[:, None, None]
    nn = n_u[:, None, None]
    pc, pr = pair_pad_flags(lens[base + ii].reshape(-1), lens[base + jj].reshape(-1), batch_size)
    pc, pr = pc.view(U, k, k - 1), pr.view(U, k, k - 1)
    ridx, tidx = mo + ii * nn + jj, mo + jj * nn + ii
    R = torch.where(pc, rmat0[ridx], rmat[ridx])
    P = torch.where(pr, rmat0[tidx], rmat[tidx])
    if which == "R":
        val = R
    elif which == "P":
        val = P
    else:
        val = 2 * P * R / (P + R)
        val = torch.nan_to_num(val, nan=0.0)
    out = torch.zeros(U, k, k, dtype=torch.float32, device=dev)
    out.scatter_(2, jj[None].expand(U, k, k - 1), val)
    return out


def mbr_scores(rmat: torch.Tensor, moff: np.ndarray, utt_off, k: int, which: str = "R"
               ) -> Tuple[np.ndarray, np.ndarray]:
    """RMBR/mbr.py:5-28 for top-k with the BERTScore utility: (argmax [U], scores float32 [U, k])."""
    lib = _lib.load()
    dev = rmat.device
    uoff = np.ascontiguousarray(utt_off, np.int32)
    n_utt = len(uoff) - 1
    if int(np.diff(uoff).min(initial=k)) < k:
        raise ValueError("every utterance needs at least k hypotheses")
    d_mo, d_uo = _dev(moff, torch.int64, dev), _dev(uoff, torch.int32, dev)
    sc = torch.empty(n_utt, k, dtype=torch.float32, device=dev)
    am = torch.empty(n_utt, dtype=torch.int32, device=dev)
    _lib.check(lib.rs_mbr_scores_bs(_lib.ptr(rmat), _lib.ptr(d_mo), _lib.ptr(d_uo), n_utt, k, WHICH[which],
                                    _lib.ptr(sc), _lib.ptr(am), _lib.stream_ptr(dev)))
    return am.cpu().numpy(), sc.cpu().numpy()


def _mbr_on_utility(util: torch.Tensor, k: int) -> Tuple[np.ndarray, np.ndarray]:
    U = util.shape[0]
    moff = np.arange(U + 1, dtype=np.int64) * k * k
    uoff = np.arange(U + 1, dtype=np.int32) * k
    return mbr_scores(util.reshape(-1), moff, uoff, k, "R")


def mbr_decode(scorer: BertScorer, nb: NBest, k: int, which: str = "R", batch_size: int = 128
               ) -> Tuple[np.ndarray, np.ndarray]:
    """RMBR/mbr.py:5-28 with ``BertScoreFunction`` (RMBR/utility_functions.py:9-22; RMBR
    config ``batch_size: 128``): (argmax [U], float32 scores [U, k])."""
    if int(np.diff(np.asarray(nb.utt_off)).min(initial=k)) < k:
        raise ValueError("every utterance needs at least k hypotheses")
    rmat, rmat0, moff = scorer.recall_matrices(nb.tokens, nb.hyp_off, nb.utt_off)
    return _mbr_on_utility(rmbr_utility(rmat, rmat0, moff, nb.hyp_off, nb.utt_off, k, which, batch_size), k)


def find_best_length(scorer: BertScorer, nb: NBest, n_best: int, which: str = "R",
                     nb_chars: NBest | None = None, batch_size: int = 128) -> Tuple[float, int, np.ndarray]:
    """RMBR/main.py:15-35 with the BERTScore utility: (best_cer, best_length, best scores).
    ``nb`` holds the model's token ids; ``nb_chars`` (same hypotheses, character symbols)
    is what the CER is measured on — ``nb`` itself when omitted.  Every k re-forms the
    reference's pair list, so the batch padding is the one each mbr_decode(k) call sees."""
    if int(np.diff(np.asarray(nb.utt_off)).min(initial=n_best)) < n_best:
        raise ValueError("every utterance needs at least n_best hypotheses")
    rmat, rmat0, moff = scorer.recall_matrices(nb.tokens, nb.hyp_off, nb.utt_off)
    nc = nb_chars if nb_chars is not None else nb
    ed_ref = ref_edits(nc, scorer.device)
    total = sum(len(r) for r in nc.refs)
    best_cer, best_len, best_sc = float("inf"), 2, None
    for k in range(2, n_best + 1):
        am, sc = _mbr_on_utility(rmbr_utility(rmat, rmat0, moff, nb.hyp_off, nb.utt_off, k, which, batch_size), k)
        arg = torch.from_numpy(am.astype(np.int32)).to(rmat.device)[None, :]
        err = float(corpus_edits(ed_ref, nb.utt_off, arg).cpu()[0]) / total
        if err < best_cer:
            best_cer, best_len, best_sc = err, k, sc
    return best_cer, best_len, best_sc
