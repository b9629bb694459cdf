"""Drop-in scorers backed by librescore (HIP, gfx950).

* ``PLLScorer`` — MLM_PLL.  ``score_nbest`` replaces the per-hypothesis accumulation of
  ``run_one_epoch(do_scoring=True)`` (MLM_PLL/main.py:73-114) over the rows of
  ``do_job`` (MLM_PLL/preprocess.py:9-30); ``masked_logprob`` replaces the row-level
  ``token_score`` (MLM_PLL/main.py:89-105) for any padded batch; ``run_one_epoch``
  mirrors the reference function's signature and ``output_score`` update.
* ``RescoreBertHIP`` — ``torch.nn.Module`` with the forward signature of
  ``RescoreBert`` (RescoreBert/model.py:13-21).

Tensors cross the C ABI as device pointers on ``torch.cuda.current_stream()``.
"""
from __future__ import annotations

import ctypes
from typing import Dict, Tuple

import numpy as np
import torch

from . import _lib
from .data import NBest
from .weights import BertShape, BERT_BASE


def _prefix_lengths(attention_mask: torch.Tensor) -> np.ndarray:
    """Row lengths of a right-padded 0/1 attention mask (``pad_sequence`` output).

    A left-padded, holed or non-binary mask would make the ragged scorers score other
    tokens than the reference's additive-mask forward, so it is rejected."""
    am = attention_mask.detach().to("cpu", torch.int64)
    if am.dim() != 2:
        raise ValueError("attention_mask must be [B, T]")
    if not bool(((am == 0) | (am == 1)).all()):
        raise ValueError("attention_mask must hold only 0 and 1")
    lens = am.sum(-1)
    pos = torch.arange(am.shape[1])[None, :]
    if not bool((am.bool() == (pos < lens[:, None])).all()):
        raise ValueError("attention_mask must be prefix ones (right padding)")
    return lens.numpy().astype(np.int32)


class BertEngine:
    """One ``rs_model`` handle: packed weights + workspace on one GPU."""

    def __init__(self, weights: Dict[str, np.ndarray], shape: BertShape = BERT_BASE,
                 heads: int = _lib.RS_HEAD_MLM, device: int | str | torch.device = 0,
                 max_rows: int = 65536, precision: str = "fp16x3"):
        if not torch.cuda.is_available():
            raise RuntimeError("librescore needs a HIP GPU (no CPU fallback)")
        self.lib = _lib.load()
        self.shape = shape
        self.device = torch.device("cuda", torch.device(device).index if not isinstance(device, int)
                                   else device)
        torch.cuda.set_device(self.device)
        cfg = _lib.RsBertCfg(shape.vocab, shape.hidden, shape.layers, shape.heads, shape.intermediate,
                             shape.max_pos, shape.type_vocab, shape.ln_eps, shape.mask_id, heads,
                             _lib.RS_PREC[precision])
        self.precision = precision
        h = ctypes.c_void_p()
        _lib.check(self.lib.rs_model_create(ctypes.byref(cfg), self.device.index, ctypes.byref(h)))
        self.handle = h
        try:
            for k, v in weights.items():
                a = np.ascontiguousarray(v, dtype=np.float32)
                shp = (ctypes.c_int64 * a.ndim)(*a.shape)
                _lib.check(self.lib.rs_model_set_tensor(self.handle, k.encode(), a.ctypes.data, 0, shp, a.ndim))
            _lib.check(self.lib.rs_model_finalize(self.handle))
            _lib.check(self.lib.rs_model_reserve(self.handle, int(max_rows)))
        except Exception:
            self.close()
            raise

    def close(self):
        if getattr(self, "handle", None):
            self.lib.rs_model_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- deferred range / timeout check (rs_model_set_sync_check, rs_check) -------------
    def set_sync_check(self, on: bool = True):
        """False: scoring calls stay asynchronous on the current stream and their non-finite /
        statistics-timeout flags accumulate until ``check()``; True (default): every call
        synchronises and raises on its own flags."""
        _lib.check(self.lib.rs_model_set_sync_check(self.handle, int(on)))

    def check(self):
        """Synchronise the current stream and raise if any deferred call flagged an error."""
        _lib.check(self.lib.rs_check(self.handle, _lib.stream_ptr(self.device)))

    # ---- profiling (HIP events per kernel kind) ----------------------------------------
    def profile(self, on: bool = True):
        _lib.check(self.lib.rs_profile_enable(self.handle, int(on)))

    def profile_read(self) -> Dict[str, Tuple[float, int, float]]:
        out = {}
        for i, name in enumerate(_lib.KINDS):
            ms, n, fl = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double()
            _lib.check(self.lib.rs_profile_read(self.handle, i, ctypes.byref(ms), ctypes.byref(n),
                                                ctypes.byref(fl)))
            out[name] = (ms.value, n.value, fl.value)
        return out

    def _dev_tokens(self, tokens) -> torch.Tensor:
        if isinstance(tokens, torch.Tensor):
            return tokens.to(self.device, torch.int32).contiguous()
        return torch.from_numpy(np.ascontiguousarray(tokens, np.int32)).to(self.device)


class PLLScorer(BertEngine):
    """MLM_PLL scorer (BertForMaskedLM head)."""

    def __init__(self, weights, shape: BertShape = BERT_BASE, device=0, max_rows: int = 65536,
                 precision: str = "fp16x3"):
        # fp16x3 (default): fp32-accurate split-fp16 operands, like the reference's fp32
        # BertForMaskedLM; "fp16" is an opt-in reduced-precision fast mode
        super().__init__(weights, shape, _lib.RS_HEAD_MLM, device, max_rows, precision)

    def score_nbest(self, tokens, hyp_off, return_rows: bool = False):
        """tokens int32 [sum T] ([CLS] w.. [SEP] per hypothesis), hyp_off int [H+1].

        Returns float64 [H] device tensor of PLL (and float32 per-row log-probs)."""
        off = np.ascontiguousarray(hyp_off, np.int32)
        n_hyp = len(off) - 1
        d_tok = self._dev_tokens(tokens)
        n_rows = int((np.diff(off) - 2).sum()) if n_hyp else 0
        pll = torch.empty(n_hyp, dtype=torch.float64, device=self.device)
        rows = torch.empty(n_rows, dtype=torch.float32, device=self.device) if return_rows else None
        _lib.check(self.lib.rs_pll_score(self.handle, _lib.ptr(d_tok), off.ctypes.data, n_hyp,
                                         _lib.ptr(pll), _lib.ptr(rows), _lib.stream_ptr(self.device)))
        return (pll, rows) if return_rows else pll

    def score(self, nb: NBest) -> np.ndarray:
        return self.score_nbest(nb.tokens, nb.hyp_off).cpu().numpy()

    def masked_logprob(self, input_ids: torch.Tensor, attention_mask: torch.Tensor,
                       labels: torch.Tensor, mask_pos) -> torch.Tensor:
        """``token_score`` of MLM_PLL/main.py:101-105 for a padded batch [B, T].

        ``attention_mask`` rows must be a prefix of ones (``pad_sequence`` output)."""
        lens = _prefix_lengths(attention_mask)
        B = input_ids.shape[0]
        mp = np.asarray([int(x) for x in mask_pos], np.int32)
        ids = input_ids.to(self.device)
        # ragged copy of the unpadded prefix of each row (device gather, no host round trip)
        T = ids.shape[1]
        keep = (torch.arange(T, device=self.device)[None, :] < torch.from_numpy(lens).to(self.device)[:, None])
        d_ids = ids[keep].to(torch.int32).contiguous()
        off = np.zeros(B + 1, np.int32)
        off[1:] = np.cumsum(lens)
        lab = labels.to(self.device)[torch.arange(B, device=self.device),
                                     torch.from_numpy(mp.astype(np.int64)).to(self.device)]
        lab = lab.to(torch.int32).contiguous()
        out = torch.empty(B, dtype=torch.float32, device=self.device)
        _lib.check(self.lib.rs_masked_logprob(self.handle, _lib.ptr(d_ids), off.ctypes.data,
                                              mp.ctypes.data, _lib.ptr(lab), B, _lib.ptr(out),
                                              _lib.stream_ptr(self.device)))
        return out

    def row_logprobs(self, rows) -> torch.Tensor:
        """``token_score`` (MLM_PLL/main.py:101-105) of every do_job row, float32 [R] (device),
        all rows in one ragged launch sequence."""
        seqs = [r["input_ids"] for r in rows]
        off = np.zeros(len(rows) + 1, np.int32)
        off[1:] = np.cumsum([len(s) for s in seqs])
        d_ids = torch.from_numpy(np.concatenate([np.asarray(s, np.int32) for s in seqs])).to(self.device)
        mp = np.asarray([r["mask_pos"] for r in rows], np.int32)
        lab = torch.from_numpy(np.asarray([r["labels"][r["mask_pos"]] for r in rows], np.int32)).to(self.device)
        out = torch.empty(len(rows), dtype=torch.float32, device=self.device)
        _lib.check(self.lib.rs_masked_logprob(self.handle, _lib.ptr(d_ids), off.ctypes.data, mp.ctypes.data,
                                              _lib.ptr(lab), len(rows), _lib.ptr(out),
                                              _lib.stream_ptr(self.device)))
        return out

    def run_one_epoch(self, rows, output_score: dict) -> dict:
        """Mirror of ``run_one_epoch(..., train_mode=False, do_scoring=True)``
        (MLM_PLL/main.py:73-114) over ``do_job`` rows (dicts with utt_id, hyp_id,
        input_ids, labels, mask_pos): scores all rows in one ragged launch sequence and
        adds them to ``output_score[utt][hyp]`` in row order (float64, like ``+=``)."""
        if not rows:
            return output_score
        for r, s in zip(rows, self.row_logprobs(rows).cpu().tolist()):
            output_score[r["utt_id"]][r["hyp_id"]] += s
        return output_score


class RescoreBertScorer(BertEngine):
    """RescoreBert scorer on ragged hypotheses (CLS head)."""

    def __init__(self, weights, shape: BertShape = BERT_BASE, device=0, max_rows: int = 65536,
                 precision: str = "fp16x3"):
        super().__init__(weights, shape, _lib.RS_HEAD_CLS, device, max_rows, precision)

    def score_nbest(self, tokens, hyp_off) -> torch.Tensor:
        off = np.ascontiguousarray(hyp_off, np.int32)
        n = len(off) - 1
        d_tok = self._dev_tokens(tokens)
        out = torch.empty(n, dtype=torch.float32, device=self.device)
        _lib.check(self.lib.rs_cls_score(self.handle, _lib.ptr(d_tok), off.ctypes.data, n,
                                         _lib.ptr(out), _lib.stream_ptr(self.device)))
        return out

    def score(self, nb: NBest) -> np.ndarray:
        return self.score_nbest(nb.tokens, nb.hyp_off).cpu().numpy()


class RescoreBertHIP(torch.nn.Module):
    """Same construction/forward contract as ``RescoreBert`` (RescoreBert/model.py:4-21).

    ``weights`` is the HF-keyed state dict (``bert.*`` + ``linear.weight/bias``) instead of
    a model name, since nothing can be fetched offline."""

    def __init__(self, weights: Dict[str, np.ndarray], shape: BertShape = BERT_BASE, device=0,
                 max_rows: int = 65536, precision: str = "fp16x3"):
        super().__init__()
        self.engine = RescoreBertScorer(weights, shape, device, max_rows, precision)

    def forward(self, input_ids: torch.Tensor, attention_mask: torch.Tensor) -> torch.Tensor:
        lens = _prefix_lengths(attention_mask)
        if (lens == 0).any():
            raise ValueError("every row needs at least one attended token")
        dev = self.engine.device
        ids = input_ids.to(dev)
        T = ids.shape[1]
        keep = torch.arange(T, device=dev)[None, :] < torch.from_numpy(lens).to(dev)[:, None]
        off = np.zeros(len(lens) + 1, np.int32)
        off[1:] = np.cumsum(lens)
        return self.engine.score_nbest(ids[keep].to(torch.int32), off)


def pll_of(weights, nb: NBest, shape: BertShape = BERT_BASE, device=0) -> np.ndarray:
    """Convenience: PLL float64 [H] of an ``NBest`` (one scorer, one call)."""
    sc = PLLScorer(weights, shape, device)
    try:
        return sc.score(nb)
    finally:
        sc.close()

