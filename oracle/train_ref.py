"""ORACLE (test infrastructure only) — torch autograd + torch.optim.AdamW restatement of the
reference's training steps, used to check the native trainer (train_api.hip).

Model: ``oracle.bert_ref.TorchBert`` (pinned against transformers via the golden fixtures)
with every parameter a leaf tensor; dropout only as explicit multipliers (``drop``: the masks
the native trainer drew, exported by ``train.dropout_keep`` and laid out by ``padded_drop``).
  * RescoreBert (RescoreBert/main.py:31-79 collate + :98-154 run_one_epoch): a batch is padded
    to its longest hypothesis (pad 0, attention mask), scores are the CLS linear head, and the
    losses are the reference's expressions (``rescorebert_loss``).
  * MLM fine-tuning (MLM_PLL/main.py:28-54 collate + :73-114 run_one_epoch): rows padded with
    id 0 and label 0, CE over every position of the padded batch (CrossEntropyLoss mean over
    B*T, the [PAD]-labelled pads included), as BertForMaskedLM computes it there.
  * ``train_rescorebert`` / ``train_mlm``: the reference's epoch loop (batches in order, a new
    AdamW every epoch, epoch loss = mean of the batch losses, dev loss without updates).
Pinned against the reference's own training runs by tests/test_oracle_golden.py (fixtures
F6/F7 of tests/golden/make_golden_train.py).
"""
from __future__ import annotations

from typing import Dict, List, Sequence

import numpy as np
import torch

from .bert_ref import TorchBert


def rescorebert_loss(sc: torch.Tensor, target, am, cer, n_best: int, method: str, md_loss_weight: float):
    """RescoreBert/main.py:104-147 on one batch (float32 tensors of the batch's rows)."""
    t = torch.as_tensor(np.asarray(target, np.float32))
    md = torch.nn.MSELoss(reduction="sum")(sc, t)
    if method == "MD":
        return md
    a = torch.as_tensor(np.asarray(am, np.float32))
    c = torch.as_tensor(np.asarray(cer, np.float32)).reshape(-1, n_best)
    mix = (sc + a).reshape(-1, n_best)
    if method == "MD_MWER":
        p = torch.softmax(mix, dim=-1)
        avg = (torch.sum(c, dim=-1) / n_best).unsqueeze(dim=-1)
        return torch.sum(torch.mul(p, c - avg)) + md_loss_weight * md
    if method == "MD_MWED":
        err = torch.softmax(c, dim=-1)
        temp = (torch.sum(mix, dim=-1) / torch.sum(c, dim=-1)).unsqueeze(dim=-1)
        q = torch.softmax(mix / temp, dim=-1)
        return torch.nn.functional.kl_div(torch.log(q), err, reduction="sum") + md_loss_weight * md
    raise ValueError(method)


class TorchTrainer:
    def __init__(self, weights: Dict[str, np.ndarray], shape, lr=1e-5, betas=(0.9, 0.999), eps=1e-8,
                 weight_decay=0.01, head: str = "cls"):
        # own copies: TorchBert wraps numpy memory and AdamW updates in place
        keep = (lambda k: not k.startswith("cls.") and not k.startswith("bert.pooler.")) if head == "cls" else \
            (lambda k: not k.startswith("linear.") and not k.startswith("bert.pooler.")
             and not k.startswith("cls.predictions.decoder."))
        self.model = TorchBert({k: np.array(v, np.float32, copy=True) for k, v in weights.items() if keep(k)}, shape)
        for t in self.model.w.values():
            t.requires_grad_(True)
        self.hp = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        self.reset_optimizer()

    def reset_optimizer(self):
        self.opt = torch.optim.AdamW(list(self.model.w.values()), **self.hp)

    def scores(self, seqs: Sequence[Sequence[int]], drop=None) -> torch.Tensor:
        T = max(len(s) for s in seqs)
        ids = torch.zeros(len(seqs), T, dtype=torch.long)
        am = torch.zeros(len(seqs), T, dtype=torch.long)
        for i, s in enumerate(seqs):
            ids[i, :len(s)] = torch.as_tensor(list(s))
            am[i, :len(s)] = 1
        return self.model.cls_score(self.model.encoder(ids, am, drop=drop))

    def step(self, seqs, target, am=None, cer=None, n_best=1, method="MD", md_loss_weight=1.0, update=True,
             drop=None):
        """update: True (backward + AdamW), False (backward only), "loss" (no backward)."""
        self.opt.zero_grad(set_to_none=False)
        with torch.set_grad_enabled(update != "loss"):
            sc = self.scores(seqs, drop)
            loss = rescorebert_loss(sc, target, am, cer, n_best, method, md_loss_weight)
            if update != "loss":
                loss.backward()
        if update is True:
            self.opt.step()
        return float(loss.detach()), sc.detach().numpy()

    def grad(self, key: str) -> np.ndarray:
        return self.model.w[key].grad.detach().numpy()

    def tensor(self, key: str) -> np.ndarray:
        return self.model.w[key].detach().numpy()

    def step_mlm(self, seqs: Sequence[Sequence[int]], labels: Sequence[Sequence[int]], update=True,
                 drop=None) -> float:
        """One reference MLM batch: pad_sequence(ids / labels, 0), attention mask, CE mean over
        all B*T positions (pads included), AdamW."""
        T = max(len(s) for s in seqs)
        x = torch.zeros(len(seqs), T, dtype=torch.long)
        am = torch.zeros(len(seqs), T, dtype=torch.long)
        lab = torch.zeros(len(seqs), T, dtype=torch.long)
        for i, (sq, lb) in enumerate(zip(seqs, labels)):
            x[i, :len(sq)] = torch.as_tensor(np.asarray(sq, np.int64))
            am[i, :len(sq)] = 1
            lab[i, :len(lb)] = torch.as_tensor(np.asarray(lb, np.int64))
        self.opt.zero_grad(set_to_none=False)
        with torch.set_grad_enabled(update != "loss"):
            logits = self.model.mlm_logits(self.model.encoder(x, am, drop=drop))
            loss = torch.nn.functional.cross_entropy(logits.view(-1, logits.shape[-1]), lab.view(-1))
            if update != "loss":
                loss.backward()
        if update is True:
            self.opt.step()
        return float(loss.detach())


def padded_drop(keep_fn, seq_lens: Sequence[int], hidden: int, heads: int, layers: int, p_hidden: float,
                p_attn: float, T: int | None = None) -> dict:
    """The native trainer's dropout masks laid out for ``TorchBert.encoder(drop=...)``.

    ``keep_fn(site, n)`` returns the keep bits (uint8 [n]) of a site in the trainer's ragged
    layout (train.h: site 0 embeddings, layer l 1 + 3l attention probabilities at
    pofs[s] + h T_s^2 + i T_s + j, 2 + 3l / 3 + 3l the residual branches at row * H + c);
    rows are the sequences' tokens back to back.  Multipliers: keep / (1 - p) in float32."""
    lens = [int(x) for x in seq_lens]
    B, Tm = len(lens), (T or max(lens))
    offs = np.concatenate([[0], np.cumsum(lens)])
    M = int(offs[-1])
    sh = np.float32(1.0 / (1.0 - p_hidden))
    sa = np.float32(1.0 / (1.0 - p_attn))

    def hid(site):
        k = keep_fn(site, M * hidden).reshape(M, hidden).astype(np.float32) * sh
        out = np.ones((B, Tm, hidden), np.float32)
        for b in range(B):
            out[b, :lens[b]] = k[offs[b]:offs[b + 1]]
        return torch.from_numpy(out)

    pofs = np.concatenate([[0], np.cumsum([heads * t * t for t in lens])])
    drop = {"emb": hid(0)}
    for i in range(layers):
        k = keep_fn(1 + 3 * i, int(pofs[-1])).astype(np.float32) * sa
        a = np.ones((B, heads, Tm, Tm), np.float32)
        for b in range(B):
            t = lens[b]
            a[b, :, :t, :t] = k[pofs[b]:pofs[b + 1]].reshape(heads, t, t)
        drop[("attn", i)] = torch.from_numpy(a)
        drop[("so", i)] = hid(2 + 3 * i)
        drop[("out", i)] = hid(3 + 3 * i)
    return drop


def _split(tokens, hyp_off):
    return [np.asarray(tokens[hyp_off[h]:hyp_off[h + 1]]).tolist() for h in range(len(hyp_off) - 1)]


def train_rescorebert(tr: TorchTrainer, train: dict, dev: dict, epochs: int, batch_size: int, n_best: int,
                      method: str, md_loss_weight: float):
    """RescoreBert/main.py:166-229's loop: ``train`` / ``dev`` = dict(seqs, pll, am, cer).
    Returns (train losses, dev losses) per epoch."""
    tl, dl = [], []
    rows = batch_size * n_best
    for _ in range(epochs):
        tr.reset_optimizer()
        for split, out, upd in ((train, tl, True), (dev, dl, "loss")):
            tot, nb = 0.0, 0
            for b0 in range(0, len(split["seqs"]), rows):
                sl = slice(b0, b0 + rows)
                loss, _ = tr.step(split["seqs"][sl], split["pll"][sl], split["am"][sl], split["cer"][sl], n_best,
                                  method, md_loss_weight, update=upd)
                tot += loss
                nb += 1
            out.append(tot / nb)
    return tl, dl


def train_mlm(tr: TorchTrainer, train: dict, dev: dict, epochs: int, batch_size: int):
    """MLM_PLL/main.py:117-161's loop over do_job rows ``dict(seqs, labels)``."""
    tl, dl = [], []
    for _ in range(epochs):
        tr.reset_optimizer()
        for split, out, upd in ((train, tl, True), (dev, dl, "loss")):
            tot, nb = 0.0, 0
            for b0 in range(0, len(split["seqs"]), batch_size):
                tot += tr.step_mlm(split["seqs"][b0:b0 + batch_size], split["labels"][b0:b0 + batch_size], update=upd)
                nb += 1
            out.append(tot / nb)
    return tl, dl
