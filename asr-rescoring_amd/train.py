"""RescoreBert distillation training and MLM fine-tuning on the GPU (SURVEY §8f item 2;
RescoreBert/main.py:82-229, MLM_PLL/main.py:73-161).

``RescoreBertTrainer`` keeps the fp32 parameters, gradients and AdamW moments of a
``RescoreBert`` (BERT encoder + ``Linear(H, 1)`` on the CLS hidden state,
RescoreBert/model.py:4-21) resident on one GPU; ``step`` runs the native training step
(``rs_train_step_cls``): forward with saved activations, the distillation loss, the backward
through head, encoder and embeddings, and one ``torch.optim.AdamW`` update.

Losses exactly as RescoreBert/main.py:104-147 computes them (``csrc/train.h``), over groups of
consecutive hypotheses (the reference's ``reshape(-1, n_best)``; ``reference_groups``):
  MD       sum_i (s_i - t_i)^2                     (MSELoss(reduction="sum"); t = mlm_pll_score)
  MD_MWER  sum_g sum_i softmax(s + am)_i (cer_i - mean_g cer) + md_loss_weight * MD
  MD_MWED  sum_g KL(softmax(cer) || softmax((s + am) / T)) + md_loss_weight * MD,
           T = sum(s + am) / sum(cer) per group, differentiated through
Pinned against the reference's own training loop (tests/golden/make_golden_train.py, F6/F7:
losses, dev scores and parameter updates after two epochs, with dropout off as the fixtures
run it).  Dropout: the reference trains under ``model.train()`` with BertConfig's defaults
(hidden_dropout_prob = attention_probs_dropout_prob = 0.1), and so do these trainers by default
— hidden dropout after the embedding LayerNorm and on both residual branches, dropout on the
attention probabilities, inverted scaling, on every training step (not on the dev-loss pass).
The masks are counter-based draws (Philox4x32-10 keyed by ``dropout_seed`` and the trainer's
dropout-step counter, ``csrc/train.h``): bitwise reproducible, and exportable
(``dropout_keep``) so the tests feed the very same masks to the CPU oracle.  torch's RNG stream
itself cannot be matched, so a reference run with dropout is matched in distribution, not bits.

``MLMTrainer`` (BertForMaskedLM, decoder tied to the word embeddings) takes the reference's
padded batches (``pad_rows``: collate of MLM_PLL/main.py:28-54 — ids and labels padded with
0, pad positions are queries but not keys) and averages the CE over every position,
[PAD]-labelled pads included, as BertForMaskedLM's loss does there.
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
                 method: str = "MD", md_loss_weight: float = 1.0, lr: float = 1e-5, betas=(0.9, 0.999),
                 eps: float = 1e-8, weight_decay: float = 0.01, hidden_dropout: float = 0.1,
                 attn_dropout: float = 0.1, dropout_seed: int = 0):
        if not torch.cuda.is_available():
            raise RuntimeError("librescore needs a HIP GPU (no CPU fallback)")
        self.lib = _lib.load()
        self.shape = shape
        self.device = torch.device("cuda", device if isinstance(device, int) else torch.device(device).index)
        torch.cuda.set_device(self.device)
        if method not in _lib.RS_LOSS:
            raise ValueError(f"unknown method {method!r} (MD, MD_MWER, MD_MWED)")
        self.method = method
        if not (0.0 <= hidden_dropout < 1.0 and 0.0 <= attn_dropout < 1.0):
            raise ValueError("dropout probabilities must be in [0, 1)")
        self.opts = _lib.RsTrainOpts(_lib.RS_LOSS[method], md_loss_weight, lr, betas[0], betas[1], eps,
                                     weight_decay, 1, hidden_dropout, attn_dropout, int(dropout_seed) & 0xFFFFFFFF)
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

    def dropout_step(self) -> int:
        """Key (dropout-step counter) of the next training step that applies dropout."""
        return int(self.lib.rs_trainer_dropout_step(self.handle))

    def set_dropout_step(self, step: int) -> None:
        _lib.check(self.lib.rs_trainer_set_dropout_step(self.handle, int(step)))

    def reset_optimizer(self):
        """A fresh AdamW (moments and step count zeroed): the reference builds its optimizer
        inside every run_one_epoch (RescoreBert/main.py:83-86, MLM_PLL/main.py:74-77)."""
        _lib.check(self.lib.rs_trainer_reset_optimizer(self.handle))

    @staticmethod
    def _update_flag(update) -> int:
        """True: backward + AdamW step; False: backward only; "loss": forward + loss only."""
        return -1 if update == "loss" else int(bool(update))

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

    def step(self, tokens, hyp_off, utt_off, target, am=None, cer=None, update=True
             ) -> Tuple[float, np.ndarray]:
        """One step on a batch (RescoreBert/main.py:98-154): ``utt_off`` groups the hypotheses
        (``reference_groups``), ``target`` = mlm_pll_score, ``am`` = hyps_am_score, ``cer`` =
        hyps_cer.  ``update``: True (backward + AdamW), False (gradients only) or "loss"
        (forward only).  Returns (loss, CLS scores before the update)."""
        hoff = np.ascontiguousarray(hyp_off, np.int32)
        uoff = np.ascontiguousarray(utt_off, np.int32)
        n = len(hoff) - 1
        dev = self.device
        d_tok = torch.as_tensor(np.ascontiguousarray(tokens, np.int32)).to(dev)
        f32 = lambda a: None if a is None else torch.as_tensor(np.asarray(a, np.float32)).to(dev)
        d_t, d_am, d_err = f32(target), f32(am), f32(cer)
        sc = torch.empty(n, dtype=torch.float32, device=dev)
        loss = torch.empty(1, dtype=torch.float32, device=dev)
        self.opts.update = self._update_flag(update)
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


def reference_groups(n_rows: int, n_best: int) -> np.ndarray:
    """Group offsets of a RescoreBert training batch: consecutive runs of ``n_best`` rows, as
    ``mix_score.reshape(-1, config.n_best)`` forms them (RescoreBert/main.py:116,132)."""
    if n_best <= 0 or n_rows % n_best:
        raise ValueError(f"batch of {n_rows} hypotheses does not reshape to (-1, {n_best})")
    return np.arange(0, n_rows + 1, n_best, dtype=np.int32)


def pad_rows(seqs: Sequence[Sequence[int]], labels: Sequence[Sequence[int]]):
    """The reference's MLM batch (collate, MLM_PLL/main.py:28-54): every row padded to the
    batch's longest with id 0 and label 0 (pad_sequence); the attention mask's zeros become
    key lengths.  Returns (ids, row_off, labels, key_len) as int32."""
    T = max(len(x) for x in seqs)
    n = len(seqs)
    ids = np.zeros((n, T), np.int32)
    lab = np.zeros((n, T), np.int32)
    klen = np.empty(n, np.int32)
    for i, (x, y) in enumerate(zip(seqs, labels)):
        ids[i, :len(x)] = x
        lab[i, :len(y)] = y
        klen[i] = len(x)
    return ids.ravel(), np.arange(0, n * T + 1, T, dtype=np.int32), lab.ravel(), klen


class MLMTrainer(_Trainer):
    """MLM fine-tuning (MLM_PLL/main.py:73-161): BertForMaskedLM, CE over every position of the
    (padded) rows, mean; AdamW.  ``key_len`` marks each row's padding (``pad_rows``); without
    it the rows are ragged and every position is real."""
    HEAD = "mlm"

    def step(self, ids, seq_off, labels, key_len=None, update=True) -> float:
        off = np.ascontiguousarray(seq_off, np.int32)
        kl = None if key_len is None else np.ascontiguousarray(key_len, np.int32)
        if kl is not None and len(kl) != len(off) - 1:
            raise ValueError("key_len needs one entry per row")
        dev = self.device
        d_ids = torch.as_tensor(np.ascontiguousarray(ids, np.int32)).to(dev)
        d_lab = torch.as_tensor(np.ascontiguousarray(labels, np.int32)).to(dev)
        loss = torch.empty(1, dtype=torch.float32, device=dev)
        self.opts.update = self._update_flag(update)
        _lib.check(self.lib.rs_train_step_mlm(self.handle, _lib.ptr(d_ids), off.ctypes.data, len(off) - 1,
                                              None if kl is None else kl.ctypes.data, _lib.ptr(d_lab),
                                              ctypes.byref(self.opts), _lib.ptr(loss), _lib.stream_ptr(dev)))
        return float(loss.item())


def rescorebert_epoch(tr: RescoreBertTrainer, tokens, hyp_off, target, am, cer, batch_size: int, n_best: int,
                      update=True) -> float:
    """One pass of RescoreBert/main.py:82-163 run_one_epoch(train=True) over the hypotheses in
    order: batches of ``batch_size * n_best`` rows (set_dataloader :71-79, shuffle False),
    groups of ``n_best`` (``reference_groups``) for MD_MWER / MD_MWED, which reshape the batch
    to (-1, n_best) (RescoreBert/main.py:116,132); MD is a plain MSELoss(sum) over the batch
    (:104-110) and takes any batch, ragged last batch and short N-best lists included;
    ``update`` True = grad_update (the caller resets AdamW first, as the reference builds it per
    call), "loss" = the dev pass.  Returns the epoch loss (mean of the batch losses)."""
    hoff = np.asarray(hyp_off, np.int64)
    n = len(hoff) - 1
    rows = batch_size * n_best
    tot, nb = 0.0, 0
    for b0 in range(0, n, rows):
        b1 = min(n, b0 + rows)
        t0, t1 = int(hoff[b0]), int(hoff[b1])
        groups = np.array([0, b1 - b0], np.int32) if tr.method == "MD" else reference_groups(b1 - b0, n_best)
        loss, _ = tr.step(np.asarray(tokens[t0:t1]), (hoff[b0:b1 + 1] - t0).astype(np.int32),
                          groups, target[b0:b1], am[b0:b1], cer[b0:b1], update=update)
        tot += loss
        nb += 1
    return tot / max(nb, 1)


def mlm_epoch(tr: MLMTrainer, seqs: Sequence[Sequence[int]], labels: Sequence[Sequence[int]], batch_size: int,
              update=True, order=None) -> float:
    """One pass of MLM_PLL/main.py:73-114 run_one_epoch (do_scoring False) over do_job rows:
    batches of ``batch_size`` rows (in ``order``, default as given), padded as the reference's
    collate pads them (``pad_rows``).  Returns the epoch loss (mean of the batch losses)."""
    idx = np.arange(len(seqs)) if order is None else np.asarray(order)
    tot, nb = 0.0, 0
    for b0 in range(0, len(idx), batch_size):
        sel = idx[b0:b0 + batch_size]
        ids, off, lab, klen = pad_rows([seqs[i] for i in sel], [labels[i] for i in sel])
        tot += tr.step(ids, off, lab, klen, update=update)
        nb += 1
    return tot / max(nb, 1)


def dropout_keep(seed: int, step: int, site: int, p: float, n: int, device=0) -> np.ndarray:
    """The keep bits (uint8 [n]) the trainer's kernels use for element e of dropout site
    ``site`` in dropout step ``step`` (``csrc/train.h``: 0 = embeddings; layer l: 1 + 3l
    attention probabilities in the saved-P layout, 2 + 3l self-output, 3 + 3l output, element
    = row * hidden + column), generated by the same device function."""
    lib = _lib.load()
    dev = torch.device("cuda", device if isinstance(device, int) else torch.device(device).index)
    out = torch.empty(max(int(n), 1), dtype=torch.uint8, device=dev)
    _lib.check(lib.rs_dropout_keep(int(seed) & 0xFFFFFFFF, int(step) & 0xFFFFFFFFFFFFFFFF, int(site), float(p), int(n),
                                   _lib.ptr(out), _lib.stream_ptr(dev)))
    return out[:int(n)].cpu().numpy()


def finetune_mlm_on_texts(weights: Dict[str, np.ndarray], sentences: Sequence[Sequence[int]],
                          shape: BertShape = BERT_BASE, steps: int = 300, batch_size: int = 64,
                          lr: float = 1e-4, seed: int = 0, device=0, dropout: float = 0.0,
                          log_every: int = 0) -> Tuple[Dict[str, np.ndarray], List[float]]:
    """MLM fine-tuning on in-domain text, then scoring with the result: the reference's
    pipeline (MLM_PLL/main.py:117-161 mlm_finetune_bert -> :184-186 scoring with that checkpoint ->
    rescore.py:25-45 fusion).  ``sentences`` are word-id lists (no [CLS]/[SEP]); their do_job rows
    (MLM_PLL/preprocess.py:9-30) are visited in a seeded permutation per epoch, ``batch_size``
    padded rows per step (collate, MLM_PLL/main.py:28-54), for ``steps`` AdamW steps.
    Deterministic (native trainer, bitwise reproducible; dropout off by default).  Returns the
    HF-keyed state dict (loadable by the scorers) and the per-step losses."""
    seqs, labels = [], []
    for s in sentences:
        h = [shape.cls_id] + [int(x) for x in s] + [shape.sep_id]
        for p in range(1, len(h) - 1):
            row = list(h)
            row[p] = shape.mask_id
            seqs.append(row)
            labels.append(h)
    tr = MLMTrainer(weights, shape, device=device, lr=lr, hidden_dropout=dropout, attn_dropout=dropout,
                    dropout_seed=seed)
    try:
        rng = np.random.Generator(np.random.PCG64(seed))
        order = np.empty(0, np.int64)
        losses: List[float] = []
        for it in range(steps):
            if len(order) < batch_size:
                order = np.concatenate([order, rng.permutation(len(seqs))])
            sel, order = order[:batch_size], order[batch_size:]
            ids, off, lab, klen = pad_rows([seqs[i] for i in sel], [labels[i] for i in sel])
            losses.append(tr.step(ids, off, lab, klen))
            if log_every and (it + 1) % log_every == 0:
                print(f"finetune step {it + 1}/{steps} loss {losses[-1]:.4f}", flush=True)
        return tr.state_dict(), losses
    finally:
        tr.close()
