"""ORACLE (test infrastructure only) — numpy/C restatement of rescore.py and RMBR (CER utility).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` may import
this.  Restated functions (reference file:line):

* ``rescore.py:47-53`` ``rescore``:  final = (1-w)*am[:, :n_best]/len + w*lm/len (fp64 numpy,
  evaluated left to right: ((1-w)*am)/len + (w*lm)/len).  Legacy variants recorded by the
  reference's own logs: ``rescore_result/MLM_PLL/rescore.log`` (``(1-w)*am + w*lm``, grid
  ``arange(0, 1.0, 0.01)``) and ``rescore_result/RMBR/BertScore/rescore_mbr_normalize.log``
  (``(1-w)*am/len + w*lm``).
* ``rescore.py:55-58`` ``get_highest_score_hyp``: ``np.argmax(axis=-1)`` (first max).
* ``rescore.py:25-45`` ``find_best_weight``: weights ``np.arange(0.0, 1.01, 0.01)``, corpus
  CER per weight, strict ``<`` keeps the first best weight.
* ``jiwer.cer`` (third-party, absent): sum of Levenshtein edits / sum of reference lengths
  (see ``oracle/levenshtein.c``); pinned by the jiwer outputs the reference records in
  ``Nbest_Align/cer.json`` (``tests/golden/jiwer_cer_pairs.json``: every value reproduced).
* ``RMBR/mbr.py:5-28`` ``mbr_decode`` + ``RMBR/utility_functions.py:28-33``: ordered pairs
  (cand = hyp_i, ref = every other hyp_j of the top-k in list order), sim = 1 - cer(ref, cand)
  as Python float64, ``torch.tensor(float32)``, ``reshape(U, k, k-1).sum(-1)`` (torch-CPU
  float32 sum order, restated in ``torch_cpu_sum_f32``), ``argmax(-1)`` (first max).
* ``RMBR/main.py:15-35`` ``find_best_length``: k = 2..n_best, strict ``<``.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import List, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "build", "liboracle_lev.so")
_lib = None

MODES = ("norm", "legacy", "am_norm")


def build_oracle_lib() -> str:
    os.makedirs(os.path.dirname(_LIB), exist_ok=True)
    src = os.path.join(_HERE, "levenshtein.c")
    if not os.path.exists(_LIB) or os.path.getmtime(_LIB) < os.path.getmtime(src):
        subprocess.check_call(["gcc", "-O2", "-shared", "-fPIC", src, "-o", _LIB])
    return _LIB


def _get_lib():
    global _lib
    if _lib is None:
        build_oracle_lib()
        _lib = ctypes.CDLL(_LIB)
        _lib.oracle_levenshtein.restype = ctypes.c_int64
        _lib.oracle_levenshtein.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32]
        _lib.oracle_pairwise.restype = None
        _lib.oracle_pairwise.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int32, ctypes.c_void_p]
    return _lib


def levenshtein(a: Sequence[int], b: Sequence[int]) -> int:
    a = np.ascontiguousarray(a, np.int32)
    b = np.ascontiguousarray(b, np.int32)
    return int(_get_lib().oracle_levenshtein(a.ctypes.data, len(a), b.ctypes.data, len(b)))


def levenshtein_py(a: Sequence, b: Sequence) -> int:
    """Pure-Python DP (small cases; an independent check of the C oracle)."""
    prev = list(range(len(b) + 1))
    for i in range(1, len(a) + 1):
        cur = [i] + [0] * len(b)
        for j in range(1, len(b) + 1):
            cur[j] = min(prev[j - 1] + (a[i - 1] != b[j - 1]), prev[j] + 1, cur[j - 1] + 1)
        prev = cur
    return prev[-1]


def corpus_cer(refs: Sequence[Sequence[int]], hyps: Sequence[Sequence[int]]) -> float:
    """jiwer.cer(list_of_refs, list_of_hyps) restated; empty reference raises like jiwer."""
    edits = 0
    total = 0
    for r, h in zip(refs, hyps):
        if len(r) == 0:
            raise ValueError("one or more references are empty strings")
        edits += levenshtein(r, h)
        total += len(r)
    return edits / total


def weight_grid(mode: str = "norm") -> np.ndarray:
    return np.arange(0.0, 1.0, 0.01) if mode == "legacy" else np.arange(0.0, 1.01, 0.01)


def fuse(weight: float, hyps_len: np.ndarray, am: np.ndarray, lm: np.ndarray,
         mode: str = "norm") -> np.ndarray:
    """rescore.py:47-53 and the two logged legacy formulas, fp64, same operation order."""
    am = np.asarray(am, np.float64)
    lm = np.asarray(lm, np.float64)
    ln = np.asarray(hyps_len)
    if mode == "norm":
        return (1 - weight) * (am) / ln + weight * (lm) / ln
    if mode == "legacy":
        return (1 - weight) * (am) + weight * (lm)
    if mode == "am_norm":
        return (1 - weight) * (am) / ln + weight * (lm)
    raise ValueError(mode)


def find_best_weight(am, lm, hyps: List[List[Sequence[int]]], refs: List[Sequence[int]],
                     n_best: int, mode: str = "norm") -> Tuple[float, float, np.ndarray]:
    """rescore.py:25-45 on dense [U, n_best] am/lm; returns (best_w, best_cer, argmax[W, U])."""
    hyps_len = np.array([[len(h) for h in utt[:n_best]] for utt in hyps])
    am = np.asarray(am, np.float64)[:, :n_best]
    best_cer, best_w = float("inf"), None
    args = []
    for w in weight_grid(mode):
        final = fuse(w, hyps_len, am, lm, mode)
        idx = np.argmax(final, axis=-1)
        args.append(idx)
        err = corpus_cer(refs, [utt[i] for utt, i in zip(hyps, idx)])
        if err < best_cer:
            best_cer, best_w = err, w
    return best_w, best_cer, np.asarray(args)


def torch_cpu_sum_f32(vals: np.ndarray) -> np.float32:
    """torch-CPU ``Tensor.sum(-1)`` float32 order for a contiguous row of n < 128 elements.

    ATen cascade_sum: n < 8 → 4 interleaved accumulators, tail into acc0, then
    acc0+acc1+acc2+acc3; n >= 8 → 8-wide vectors summed with 4 vector accumulators,
    scalar tail, then the 8 lanes added to the tail sequentially.  Verified bit-exact
    against torch 2.10 for n = 1..99 in this container (tests/test_oracle_rescore.py).
    """
    v = np.asarray(vals, np.float32)
    F = np.float32

    def row_sum(items):
        n = len(items)
        sz = n // 4
        acc = []
        for k in range(4):
            a = np.zeros_like(items[0]) if n else F(0)
            for i in range(sz):
                a = (a + items[i * 4 + k]).astype(F)
            acc.append(a)
        for i in range(sz * 4, n):
            acc[0] = (acc[0] + items[i]).astype(F)
        for k in range(1, 4):
            acc[0] = (acc[0] + acc[k]).astype(F)
        return acc[0]

    n = len(v)
    if n == 0:
        return F(0)
    if n < 8:
        return F(row_sum([v[j] for j in range(n)]))
    nv = n // 8
    va = row_sum([v[i * 8:(i + 1) * 8] for i in range(nv)])
    fin = F(0)
    for i in range(nv * 8, n):
        fin = F(fin + v[i])
    for k in range(8):
        fin = F(fin + va[k])
    return fin


def mbr_decode(k: int, all_hyps: List[List[Sequence[int]]]) -> Tuple[np.ndarray, np.ndarray]:
    """RMBR/mbr.py:5-28 with CerScoreFunction (RMBR/utility_functions.py:28-33).

    Returns (argmax int64 [U], scores float32 [U, k])."""
    U = len(all_hyps)
    scores = np.zeros((U, k), np.float32)
    for u, hyps in enumerate(all_hyps):
        for i in range(k):
            sims = []
            for j in list(range(0, i)) + list(range(i + 1, k)):
                ref, cand = hyps[j], hyps[i]
                c = levenshtein(ref, cand) / len(ref)          # jiwer.cer(ref, cand)
                sims.append(np.float32(1 - c))                  # torch.tensor(float32)
            scores[u, i] = torch_cpu_sum_f32(np.asarray(sims, np.float32))
    return np.argmax(scores, axis=-1), scores


def find_best_length(n_best: int, refs, hyps) -> Tuple[float, int, np.ndarray]:
    """RMBR/main.py:15-35."""
    best_cer, best_len, best_scores = float("inf"), 2, None
    for k in range(2, n_best + 1):
        idx, sc = mbr_decode(k, hyps)
        err = corpus_cer(refs, [h[i] for h, i in zip(hyps, idx)])
        if err < best_cer:
            best_cer, best_len, best_scores = err, k, sc
    return best_cer, best_len, best_scores
