"""RescoreBert distillation training on the GPU (RescoreBert/main.py:104-229).

``RescoreBertTrainer`` keeps the fp32 parameters, gradients and AdamW moments of a
``RescoreBert`` (BERT encoder + ``Linear(H, 1)`` on the CLS hidden state,
RescoreBert/model.py:4-21) resident on one GPU; ``step`` runs the native training step
(``rs_train_step_cls``): forward with saved activations, the distillation loss, the backward
through head, encoder and embeddings, and one ``torch.optim.AdamW`` update.

Losses (restated from the RescoreBERT paper; the reference's loss code was not consulted
this round, so their parity is unpinned — the backward and the optimizer are checked against
torch autograd + ``torch.optim.AdamW`` on the same loss, tests/test_gpu_train.py):
  MD       mean_i (s_i - t_i)^2, t_i = the hypothesis' MLM PLL (the teacher)
  MD_MWER  MD + lambda * mean_u sum_i softmax(am + s)_i (err_i - mean err)
  MD_MWED  MD + lambda * mean_u -sum_i softmax(-err)_i log softmax((am + s) / tau)_i
Dropout is not applied (the step is deterministic and bitwise reproducible).
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib
from .weights import BertShape, BERT_BASE


def param_shapes(shape: BertShape, head: str = "cls") -> Dict[str, Tuple[int, ...]]:
    """HF keys and shapes a trainer owns: RescoreBert without the unused pooler ("cls"), or
    BertForMaskedLM with its decoder tied to the word embeddings ("mlm")."""
    H, F = shape.hidden, shape.intermediate
    e = "bert.embeddings."
    out = {e + "word_embeddings.weight": (shape.vocab, H), e + "position_embeddings.weight": (shape.max_pos, H),
           e + "token_type_embeddings.weight": (shape.type_vocab, H), e + "LayerNorm.weight": (H,),
           e + "LayerNorm.bias": (H,)}
    for i in range(shape.layers):
        p = f"bert.encoder.layer.{i}."
        for n in ("query", "key", "value"):
            out[p + f"attention.self.{n}.weight"] = (H, H)
            out[p + f"attention.self.{n}.bias"] = (H,)
        out.update({p + "attention.output.dense.weight": (H, H), p + "attention.output.dense.bias": (H,),
                    p + "attention.output.LayerNorm.weight": (H,), p + "attention.output.LayerNorm.bias": (H,),
                    p + "intermediate.dense.weight": (F, H), p + "intermediate.dense.bias": (F,),
                    p + "output.dense.weight": (H, F), p + "output.dense.bias": (H,),
                    p + "output.LayerNorm.weight": (H,), p + "output.LayerNorm.bias": (H,)})
    if head == "mlm":
        c = "cls.predictions."
        out.update({c + "transform.dense.weight": (H, H), c + "transform.dense.bias": (H,),
                    c + "transform.LayerNorm.weight": (H,), c + "transform.LayerNorm.bias": (H,),
                    c + "bias": (shape.vocab,)})
    else:
        out["linear.weight"] = (1, H)
        out["linear.bias"] = (1,)
    return out


class _Trainer:
    HEAD = "cls"

    def __init__(self, weights: Dict[str, np.ndarray], shape: BertShape = BERT_BASE, device=0,
                 loss: str = "MD", lam: float = 1.0, lr: float = 1e-5, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.01):
        if not torch.cuda.is_available():
            raise RuntimeError("librescore needs a HIP GPU (no CPU fallback)")
        self.lib = _lib.load()
        self.shape = shape
        self.device = torch.device("cuda", device if isinstance(device, int) else torch.device(device).index)
        torch.cuda.set_device(self.device)
        self.opts = _lib.RsTrainOpts(_lib.RS_LOSS[loss], lam, lr, betas[0], betas[1], eps, weight_decay, 1)
        self.shapes = param_shapes(shape, self.HEAD)
        self.extra = {k: np.asarray(v) for k, v in weights.items()
                      if k.startswith("bert.pooler.") or (self.HEAD == "mlm" and k.startswith("cls.predictions.decoder."))}
        heads = _lib.RS_HEAD_CLS if self.HEAD == "cls" else _lib.RS_HEAD_MLM
        cfg = _lib.RsBertCfg(shape.vocab, shape.hidden, shape.layers, shape.heads, shape.intermediate,
                             shape.max_pos, shape.type_vocab, shape.ln_eps, shape.mask_id, heads, 0)
        h = ctypes.c_void_p()
        _lib.check(self.lib.rs_trainer_create(ctypes.byref(cfg), self.device.index, ctypes.byref(h)))
        self.handle = h
        try:
            for k, v in weights.items():
                if k not in self.shapes:          # e.g. an MLM head when initialising from BertForMaskedLM
                    continue
                a = np.ascontiguousarray(v, dtype=np.float32)
                shp = (ctypes.c_int64 * a.ndim)(*a.shape)
                _lib.check(self.lib.rs_trainer_set_tensor(self.handle, k.encode(), a.ctypes.data, 0, shp, a.ndim))
            _lib.check(self.lib.rs_trainer_finalize(self.handle))
        except Exception:
            self.close()
            raise

    def close(self):
        if getattr(self, "handle", None):
            self.lib.rs_trainer_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset_optimizer(self):
        _lib.check(self.lib.rs_trainer_reset_optimizer(self.handle))

    def _get(self, fn, key: str) -> np.ndarray:
        shp = self.shapes[key]
        out = np.empty(shp, np.float32)
        _lib.check(fn(self.handle, key.encode(), out.ctypes.data, out.size))
        return out

    def tensor(self, key: str) -> np.ndarray:
        return self._get(self.lib.rs_trainer_get_tensor, key)

    def grad(self, key: str) -> np.ndarray:
        return self._get(self.lib.rs_trainer_get_grad, key)

    def state_dict(self) -> Dict[str, np.ndarray]:
        """HF-keyed weights (what the scorers load); the pooler passes through unchanged, the
        tied MLM decoder weight is the trained word-embedding matrix."""
        sd = {k: self.tensor(k) for k in self.shapes}
        sd.update(self.extra)
        if "cls.predictions.decoder.weight" in sd:
            sd["cls.predictions.decoder.weight"] = sd["bert.embeddings.word_embeddings.weight"]
        if "cls.predictions.decoder.bias" in sd:
            sd["cls.predictions.decoder.bias"] = sd["cls.predictions.bias"]
        return sd


class RescoreBertTrainer(_Trainer):
    HEAD = "cls"

    def step(self, tokens, hyp_off, utt_off, target, am=None, err=None, update: bool = True
             ) -> Tuple[float, np.ndarray]:
        """One training step on a batch of utterances; returns (loss, CLS scores before the update)."""
        hoff = np.ascontiguousarray(hyp_off, np.int32)
        uoff = np.ascontiguousarray(utt_off, np.int32)
        n = len(hoff) - 1
        dev = self.device
        d_tok = torch.as_tensor(np.ascontiguousarray(tokens, np.int32)).to(dev)
        f32 = lambda a: None if a is None else torch.as_tensor(np.asarray(a, np.float32)).to(dev)
        d_t, d_am, d_err = f32(target), f32(am), f32(err)
        sc = torch.empty(n, dtype=torch.float32, device=dev)
        loss = torch.empty(1, dtype=torch.float32, device=dev)
        self.opts.update = int(update)
        _lib.check(self.lib.rs_train_step_cls(self.handle, _lib.ptr(d_tok), hoff.ctypes.data, n, uoff.ctypes.data,
                                              len(uoff) - 1, _lib.ptr(d_t), _lib.ptr(d_am), _lib.ptr(d_err),
                                              ctypes.byref(self.opts), _lib.ptr(sc), _lib.ptr(loss),
                                              _lib.stream_ptr(dev)))
        return float(loss.item()), sc.cpu().numpy()


def do_job_rows(hyps: Sequence[Sequence[int]], mask_id: int = 103):
    """MLM_PLL/preprocess.py:9-30 rows of [CLS] w.. [SEP] sequences: one [MASK] per word
    position; labels = the unmasked sequence.  Returns (ids, seq_off, labels) ragged int32."""
    ids, labels, off = [], [], [0]
    for h in hyps:
        h = list(h)
        for p in range(1, len(h) - 1):
            row = h.copy()
            row[p] = mask_id
            ids.extend(row)
            labels.extend(h)
            off.append(off[-1] + len(h))
    return np.asarray(ids, np.int32), np.asarray(off, np.int32), np.asarray(labels, np.int32)


class MLMTrainer(_Trainer):
    """MLM fine-tuning (MLM_PLL/main.py:117-161): BertForMaskedLM, CE over every real position
    of each row (mean), AdamW.  Rows are ragged (no padding positions in the loss)."""
    HEAD = "mlm"

    def step(self, ids, seq_off, labels, update: bool = True) -> float:
        off = np.ascontiguousarray(seq_off, np.int32)
        dev = self.device
        d_ids = torch.as_tensor(np.ascontiguousarray(ids, np.int32)).to(dev)
        d_lab = torch.as_tensor(np.ascontiguousarray(labels, np.int32)).to(dev)
        loss = torch.empty(1, dtype=torch.float32, device=dev)
        self.opts.update = int(update)
        _lib.check(self.lib.rs_train_step_mlm(self.handle, _lib.ptr(d_ids), off.ctypes.data, len(off) - 1,
                                              _lib.ptr(d_lab), ctypes.byref(self.opts), _lib.ptr(loss),
                                              _lib.stream_ptr(dev)))
        return float(loss.item())
