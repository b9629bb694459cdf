"""Levenshtein alignment with backtrace on the GPU (SURVEY §8f item 4;
espnet_data/preprocess/align.py:5-97 ``levenshtein_distance_alignment``, used by
Nbest_Align/preprocess.py:92-108 and CorrectBart/get_feature.py:111-127 to align N-best
hypotheses token by token).

``levenshtein_distance_alignment(ref, hyp)`` keeps the reference's call shape and output
(``[ref_aligned, hyp_aligned, ops]`` with ``"*"`` gaps and ops U / S / I / D);
``align_batch(pairs)`` aligns many pairs in one launch of the ``rs_align`` kernel (one wave per
pair, anti-diagonal wavefront, csrc/k_align.hip).  Tokens may be any hashable values (CJK
characters, words): they are mapped to int32 ids on the host.  No CPU fallback.
"""
from __future__ import annotations

import ctypes
from typing import Hashable, List, Sequence, Tuple

import numpy as np
import torch

from . import _lib

OPS = ("U", "S", "I", "D")      # RS_AL_U / _S / _I / _D
GAP = "*"


def _encode(pairs: Sequence[Tuple[Sequence[Hashable], Sequence[Hashable]]]):
    vocab: dict = {}
    ids = lambda seq: [vocab.setdefault(t, len(vocab)) for t in seq]      # noqa: E731
    ref = [ids(r) for r, _ in pairs]
    hyp = [ids(h) for _, h in pairs]
    return ref, hyp


def align_ids(ref: List[List[int]], hyp: List[List[int]], device=0):
    """Raw kernel call on int token ids: (ops int8, ref_idx int32, hyp_idx int32, out_off int64,
    n int32) as numpy arrays, pair p's alignment at out_off[p] .. out_off[p] + n[p]."""
    if len(ref) != len(hyp):
        raise ValueError("ref and hyp lists differ in length")
    if not torch.cuda.is_available():
        raise RuntimeError("librescore needs a HIP GPU (no CPU fallback)")
    lib = _lib.load()
    dev = torch.device("cuda", device)
    P = len(ref)
    lr = np.asarray([len(r) for r in ref], np.int64)
    lh = np.asarray([len(h) for h in hyp], np.int64)
    cat = lambda xs: np.asarray([t for x in xs for t in x], np.int32)     # noqa: E731
    off = lambda ls: np.concatenate([[0], np.cumsum(ls)]).astype(np.int32)  # noqa: E731
    lab_off = np.concatenate([[0], np.cumsum((lr + 1) * (lh + 1))]).astype(np.int64)
    out_off = np.concatenate([[0], np.cumsum(lr + lh)]).astype(np.int64)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)       # noqa: E731
    pad = lambda a: np.append(a, np.zeros(1, np.int32))                   # noqa: E731 (no empty buffers)
    d_ref, d_roff, d_hyp, d_hoff = T(pad(cat(ref))), T(off(lr)), T(pad(cat(hyp))), T(off(lh))
    assert d_ref.dtype == d_hyp.dtype == d_roff.dtype == torch.int32
    d_loff, d_ooff = T(lab_off), T(out_off)
    n_out = max(int(out_off[-1]), 1)
    d_lab = torch.empty(max(int(lab_off[-1]), 1), dtype=torch.uint8, device=dev)
    d_ops = torch.empty(n_out, dtype=torch.int8, device=dev)
    d_ri = torch.empty(n_out, dtype=torch.int32, device=dev)
    d_hi = torch.empty(n_out, dtype=torch.int32, device=dev)
    d_n = torch.empty(max(P, 1), dtype=torch.int32, device=dev)
    max_len = int(max(lr.max(initial=0), lh.max(initial=0)))
    _lib.check(lib.rs_align(_lib.ptr(d_ref), _lib.ptr(d_roff), _lib.ptr(d_hyp), _lib.ptr(d_hoff), P,
                            _lib.ptr(d_loff), _lib.ptr(d_lab), _lib.ptr(d_ooff), _lib.ptr(d_ops), _lib.ptr(d_ri),
                            _lib.ptr(d_hi), _lib.ptr(d_n), max_len, _lib.stream_ptr(dev)))
    return (d_ops.cpu().numpy(), d_ri.cpu().numpy(), d_hi.cpu().numpy(), out_off, d_n.cpu().numpy()[:P])


def align_batch(pairs: Sequence[Tuple[Sequence[Hashable], Sequence[Hashable]]], device=0) -> List[List[list]]:
    """[levenshtein_distance_alignment(ref, hyp) for (ref, hyp) in pairs], one kernel launch."""
    ref, hyp = _encode(pairs)
    ops, ri, hi, out_off, n = align_ids(ref, hyp, device)
    res = []
    for p, (r, h) in enumerate(pairs):
        a, b = int(out_off[p]), int(out_off[p]) + int(n[p])
        res.append([[r[k] if k >= 0 else GAP for k in ri[a:b]], [h[k] if k >= 0 else GAP for k in hi[a:b]],
                    [OPS[o] for o in ops[a:b]]])
    return res


def levenshtein_distance_alignment(ref: Sequence[Hashable], hyp: Sequence[Hashable], device=0) -> List[list]:
    """espnet_data/preprocess/align.py:5-97 on one pair: [ref_aligned, hyp_aligned, ops]."""
    return align_batch([(ref, hyp)], device)[0]
