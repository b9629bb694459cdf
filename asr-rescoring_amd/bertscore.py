"""BERTScore MBR utility on the GPU.

The reference's ``BertScoreFunction`` (RMBR/utility_functions.py:9-22) calls
``bert_score.score(cands, refs, lang="zh")``: bert-base-chinese truncated to its first 8
encoder layers, ``idf=False``, no baseline rescaling.  ``bert_score`` is not installed (and
the model is fetched by name), so this module implements the library's published algorithm
on the HIP path:

* ``BertScorer.embed`` — ``get_bert_embedding`` / ``bert_encode``: the last hidden state of
  the truncated encoder for every token, L2-normalised as ``greedy_cos_idf`` does first
  (``rs_token_embed``).
* ``BertScorer.recall_matrix`` — ``greedy_cos_idf`` for every ordered pair (cand i, ref j)
  of each utterance's hypotheses in one fused MFMA kernel (``rs_bertscore_recall``):
  R(i|j), with P(i|j) = R(j|i) and F = 2PR / (P + R).
* ``BertScorer.score(cands, refs)`` — ``bert_score.score``'s (P, R, F) for aligned lists.
* ``mbr_decode`` / ``find_best_length`` — RMBR/mbr.py:5-28 and RMBR/main.py:15-35 with this
  utility (``rs_mbr_scores_bs``; same float32 summation order and first-max argmax as the
  CER utility in ``rerank``).

Difference from bert_score, by construction: bert_score pads a batch of pairs and multiplies
the cosine matrix by the pad masks, so a padded position contributes a cosine of 0 to the max;
here the max runs over the real tokens only.  The two agree whenever a token's best cosine is
non-negative.
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
                 device=0, max_rows: int = 65536, precision: str = "fp16"):
        num_layers = min(num_layers, shape.layers)
        sh = dataclasses.replace(shape, layers=num_layers)
        super().__init__(truncate_weights(weights, num_layers), sh, _lib.RS_HEAD_EMB, device, max_rows,
                         precision)

    def embed(self, tokens, hyp_off) -> torch.Tensor:
        """fp16 [sum T, H]: L2-normalised last hidden state of every token."""
        off = np.ascontiguousarray(hyp_off, np.int32)
        d_tok = self._dev_tokens(tokens)
        out = torch.empty(int(off[-1]) if len(off) else 0, self.shape.hidden, dtype=torch.float16,
                          device=self.device)
        _lib.check(self.lib.rs_token_embed(self.handle, _lib.ptr(d_tok), off.ctypes.data, len(off) - 1,
                                           _lib.ptr(out), _lib.stream_ptr(self.device)))
        return out

    def recall_matrix(self, tokens, hyp_off, utt_off) -> Tuple[torch.Tensor, np.ndarray]:
        """Concatenated n_u x n_u float32 blocks R[i, j] = R(cand i | ref j), and their offsets."""
        hoff = np.ascontiguousarray(hyp_off, np.int32)
        uoff = np.ascontiguousarray(utt_off, np.int32)
        n_u = np.diff(uoff).astype(np.int64)
        moff = np.zeros(len(uoff), np.int64)
        moff[1:] = np.cumsum(n_u * n_u)
        d_tok = self._dev_tokens(tokens)
        rmat = torch.empty(int(moff[-1]), dtype=torch.float32, device=self.device)
        _lib.check(self.lib.rs_bertscore_recall(self.handle, _lib.ptr(d_tok), hoff.ctypes.data, uoff.ctypes.data,
                                                len(uoff) - 1, _lib.ptr(rmat), _lib.stream_ptr(self.device)))
        return rmat, moff

    def score(self, cands: Sequence[Sequence[int]], refs: Sequence[Sequence[int]]
              ) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """``bert_score.score(cands, refs)`` on token ids ([CLS] w.. [SEP] each): (P, R, F)."""
        if len(cands) != len(refs):
            raise ValueError("cands and refs differ in length")
        seqs = [s for pair in zip(cands, refs) for s in pair]
        hoff = np.zeros(len(seqs) + 1, np.int32)
        hoff[1:] = np.cumsum([len(s) for s in seqs])
        toks = np.concatenate([np.asarray(s, np.int32) for s in seqs]) if seqs else np.zeros(0, np.int32)
        uoff = np.arange(0, len(seqs) + 1, 2, dtype=np.int32)
        rmat, _ = self.recall_matrix(toks, hoff, uoff)
        r = rmat.view(-1, 2, 2).cpu().numpy()
        R, P = r[:, 0, 1], r[:, 1, 0]          # (cand 0 | ref 1) and its transpose
        with np.errstate(invalid="ignore", divide="ignore"):
            F = (np.float32(2) * P * R / (P + R)).astype(np.float32)
        F[np.isnan(F)] = 0.0
        return P, R, F


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


def mbr_decode(scorer: BertScorer, nb: NBest, k: int, which: str = "R") -> Tuple[np.ndarray, np.ndarray]:
    rmat, moff = scorer.recall_matrix(nb.tokens, nb.hyp_off, nb.utt_off)
    return mbr_scores(rmat, moff, nb.utt_off, k, which)


def find_best_length(scorer: BertScorer, nb: NBest, n_best: int, which: str = "R",
                     nb_chars: NBest | None = None) -> Tuple[float, int, np.ndarray]:
    """RMBR/main.py:15-35 with the BERTScore utility: (best_cer, best_length, best scores).
    ``nb`` holds the model's token ids; ``nb_chars`` (same hypotheses, character symbols)
    is what the CER is measured on — ``nb`` itself when omitted."""
    rmat, moff = scorer.recall_matrix(nb.tokens, nb.hyp_off, nb.utt_off)
    nc = nb_chars if nb_chars is not None else nb
    ed_ref = ref_edits(nc, scorer.device)
    total = sum(len(r) for r in nc.refs)
    best_cer, best_len, best_sc = float("inf"), 2, None
    for k in range(2, n_best + 1):
        am, sc = mbr_scores(rmat, moff, nb.utt_off, k, which)
        arg = torch.from_numpy(am.astype(np.int32)).to(rmat.device)[None, :]
        err = float(corpus_edits(ed_ref, nb.utt_off, arg).cpu()[0]) / total
        if err < best_cer:
            best_cer, best_len, best_sc = err, k, sc
    return best_cer, best_len, best_sc
