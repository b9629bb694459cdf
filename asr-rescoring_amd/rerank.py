"""AM/LM fusion, argmax, corpus CER and RMBR (CER utility) on the GPU.

Host mirrors of the reference functions (same names, argument meaning, tie rules):

* ``find_best_weight`` — rescore.py:25-45 (101-weight grid, strict ``<`` keeps the first
  best weight); the whole grid is one ``rs_fuse_rerank`` launch and the corpus CER of every
  weight is one ``rs_corpus_edits`` launch over a per-hypothesis ``ed(ref, hyp)`` table
  (``rs_ref_edit``), exactly Σ edits / Σ ref chars as ``jiwer.cer`` computes it.
* ``fuse_rerank`` — ``rescore`` + ``get_highest_score_hyp`` (rescore.py:47-58).
* ``mbr_decode`` / ``find_best_length`` — RMBR/mbr.py:5-28, RMBR/main.py:15-35 with
  ``CerScoreFunction``; the pairwise edit matrix is computed once and reused for every k.

Inputs are ``NBest`` (token/char ids); "characters" are symbols, as jiwer's CER splits text
into characters (CJK: one token per character).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np
import torch

from . import _lib
from .data import NBest

# Edit-distance kernels (csrc/k_rerank.hip): exact for strings of up to RS_MAX_EDIT symbols
MAX_EDIT_LEN = 16384


def _dev(a, dtype, device):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype).to(device)


def weight_grid(mode: str = "norm") -> np.ndarray:
    """rescore.py:37 (np.arange(0.0, 1.01, 0.01)); the legacy log used arange(0, 1.0, 0.01)."""
    return np.arange(0.0, 1.0, 0.01) if mode == "legacy" else np.arange(0.0, 1.01, 0.01)


def _strings(nb: NBest):
    """Hypothesis words only ([CLS]/[SEP] stripped), flat int32 + offsets (vectorised)."""
    off = np.asarray(nb.hyp_off, np.int64)
    keep = np.ones(len(nb.tokens), bool)
    if nb.n_hyp:
        keep[off[:-1]] = False           # [CLS]
        keep[off[1:] - 1] = False        # [SEP]
    flat = np.ascontiguousarray(nb.tokens[keep], np.int32)
    soff = np.zeros(nb.n_hyp + 1, np.int32)
    soff[1:] = np.cumsum(np.diff(off) - 2)
    return flat, soff


def ref_edits(nb: NBest, device=0) -> torch.Tensor:
    """int32 [H] = Levenshtein(ref_u, hyp_h) for every hypothesis (device)."""
    lib = _lib.load()
    dev = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
    flat, soff = _strings(nb)
    if any(len(r) == 0 for r in nb.refs):
        raise ValueError("one or more references are empty strings")   # jiwer behaviour
    rflat = np.concatenate(nb.refs).astype(np.int32)
    roff = np.zeros(nb.n_utt + 1, np.int32)
    roff[1:] = np.cumsum([len(r) for r in nb.refs])
    if max(int(np.diff(soff).max(initial=0)), int(np.diff(roff).max(initial=0))) > MAX_EDIT_LEN:
        raise ValueError(f"strings longer than {MAX_EDIT_LEN} symbols are not supported")
    d_c, d_so, d_uo = _dev(flat, torch.int32, dev), _dev(soff, torch.int32, dev), _dev(nb.utt_off, torch.int32, dev)
    d_rc, d_ro = _dev(rflat, torch.int32, dev), _dev(roff, torch.int32, dev)
    out = torch.empty(nb.n_hyp, dtype=torch.int32, device=dev)
    _lib.check(lib.rs_ref_edit(_lib.ptr(d_c), _lib.ptr(d_so), _lib.ptr(d_uo), _lib.ptr(d_rc), _lib.ptr(d_ro),
                               nb.n_utt, _lib.ptr(out), _lib.stream_ptr(dev)))
    return out


def fuse_rerank(am, lm, hyp_len, utt_off, weights, mode: str = "norm", n_best: int = 1 << 30,
                device=0) -> torch.Tensor:
    """argmax int32 [W, U] of the fused scores for every weight (device)."""
    lib = _lib.load()
    dev = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
    am_d = am if isinstance(am, torch.Tensor) else _dev(am, torch.float64, dev)
    lm_d = lm if isinstance(lm, torch.Tensor) else _dev(lm, torch.float64, dev)
    am_d, lm_d = am_d.to(dev, torch.float64).contiguous(), lm_d.to(dev, torch.float64).contiguous()
    ln = _dev(hyp_len, torch.int32, dev)
    uo = _dev(utt_off, torch.int32, dev)
    w = _dev(np.asarray(weights, np.float64), torch.float64, dev)
    n_utt = len(utt_off) - 1
    out = torch.empty(len(weights), n_utt, dtype=torch.int32, device=dev)
    _lib.check(lib.rs_fuse_rerank(_lib.ptr(am_d), _lib.ptr(lm_d), _lib.ptr(ln), _lib.ptr(uo), n_utt,
                                  min(int(n_best), 2**31 - 1), _lib.ptr(w), len(weights), _lib.RS_FUSE[mode],
                                  _lib.ptr(out), _lib.stream_ptr(dev)))
    return out


def corpus_edits(ed_ref: torch.Tensor, utt_off, argmax: torch.Tensor, device=0) -> torch.Tensor:
    lib = _lib.load()
    dev = argmax.device
    uo = _dev(utt_off, torch.int32, dev)
    W, U = argmax.shape
    out = torch.empty(W, dtype=torch.int64, device=dev)
    _lib.check(lib.rs_corpus_edits(_lib.ptr(ed_ref), _lib.ptr(uo), _lib.ptr(argmax.contiguous()), U, W,
                                   _lib.ptr(out), _lib.stream_ptr(dev)))
    return out


def find_best_weight(nb: NBest, lm, n_best: int = 10, mode: str = "norm", device=0
                     ) -> Tuple[float, float, np.ndarray, np.ndarray]:
    """rescore.py:25-45: returns (best_weight, best_cer, argmax [W, U], cer [W])."""
    grid = weight_grid(mode)
    lens = nb.hyp_len()
    arg = fuse_rerank(nb.am, lm, lens, nb.utt_off, grid, mode, n_best, device)
    ed = ref_edits(nb, device)
    edits = corpus_edits(ed, nb.utt_off, arg, device).cpu().numpy()
    total = sum(len(r) for r in nb.refs)
    cers = edits / total
    best_i, best = 0, float("inf")
    for i, c in enumerate(cers):            # strict '<' keeps the first best (rescore.py:41)
        if c < best:
            best, best_i = c, i
    return float(grid[best_i]), float(best), arg.cpu().numpy(), cers


def pairwise_edit(nb: NBest, device=0) -> Tuple[torch.Tensor, np.ndarray]:
    """Concatenated n_u x n_u int32 matrices and their int64 offsets."""
    lib = _lib.load()
    dev = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
    flat, soff = _strings(nb)
    n_u = np.diff(nb.utt_off).astype(np.int64)
    moff = np.zeros(nb.n_utt + 1, np.int64)
    moff[1:] = np.cumsum(n_u * n_u)
    if len(soff) > 1 and int(np.diff(soff).max()) > MAX_EDIT_LEN:
        raise ValueError(f"strings longer than {MAX_EDIT_LEN} symbols are not supported")
    d_c, d_so = _dev(flat, torch.int32, dev), _dev(soff, torch.int32, dev)
    d_uo, d_mo = _dev(nb.utt_off, torch.int32, dev), _dev(moff, torch.int64, dev)
    ed = torch.empty(int(moff[-1]), dtype=torch.int32, device=dev)
    _lib.check(lib.rs_pairwise_edit(_lib.ptr(d_c), _lib.ptr(d_so), _lib.ptr(d_uo), _lib.ptr(d_mo), nb.n_utt,
                                    int(n_u.max(initial=0)), _lib.ptr(ed), _lib.stream_ptr(dev)))
    return ed, moff


def mbr_scores(nb: NBest, k: int, ed: torch.Tensor, moff: np.ndarray, device=0
               ) -> Tuple[np.ndarray, np.ndarray]:
    """RMBR/mbr.py:5-28 for top-k: (argmax int [U], scores float32 [U, k])."""
    lib = _lib.load()
    dev = ed.device
    if int(np.diff(nb.utt_off).min(initial=k)) < k:
        raise ValueError("every utterance needs at least k hypotheses")
    lens = nb.hyp_len()
    if (lens == 0).any():
        raise ValueError("one or more references are empty strings")   # jiwer on an empty hyp_j
    d_mo, d_uo = _dev(moff, torch.int64, dev), _dev(nb.utt_off, torch.int32, dev)
    d_len = _dev(lens, torch.int32, dev)
    sc = torch.empty(nb.n_utt, k, dtype=torch.float32, device=dev)
    am = torch.empty(nb.n_utt, dtype=torch.int32, device=dev)
    _lib.check(lib.rs_mbr_scores(_lib.ptr(ed), _lib.ptr(d_mo), _lib.ptr(d_uo), _lib.ptr(d_len), nb.n_utt, k,
                                 _lib.ptr(sc), _lib.ptr(am), _lib.stream_ptr(dev)))
    return am.cpu().numpy(), sc.cpu().numpy()


def mbr_decode(nb: NBest, k: int, device=0) -> Tuple[np.ndarray, np.ndarray]:
    ed, moff = pairwise_edit(nb, device)
    return mbr_scores(nb, k, ed, moff, device)


def find_best_length(nb: NBest, n_best: int, device=0) -> Tuple[float, int, np.ndarray]:
    """RMBR/main.py:15-35: (best_cer, best_length, best scores [U, k])."""
    ed, moff = pairwise_edit(nb, device)
    ed_ref = ref_edits(nb, device)
    total = sum(len(r) for r in nb.refs)
    best_cer, best_len, best_sc = float("inf"), 2, None
    for k in range(2, n_best + 1):
        am, sc = mbr_scores(nb, k, ed, moff, device)
        arg = torch.from_numpy(am.astype(np.int32)).to(ed.device)[None, :]
        err = float(corpus_edits(ed_ref, nb.utt_off, arg).cpu()[0]) / total
        if err < best_cer:
            best_cer, best_len, best_sc = err, k, sc
    return best_cer, best_len, best_sc


def argmax_words(nb: NBest, idx: Sequence[int]) -> List[np.ndarray]:
    return [nb.hyp_words(nb.utt_off[u] + int(i)) for u, i in enumerate(idx)]
