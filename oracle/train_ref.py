"""ORACLE (test infrastructure only) — torch autograd + torch.optim.AdamW restatement of a
RescoreBert distillation training step, used to check the native trainer (train_api.hip).

Model: ``oracle.bert_ref.TorchBert`` (pinned against the reference's own RescoreBert via the
golden fixtures) with every parameter a leaf tensor; a batch is padded to its longest
hypothesis (``RescoreBert/main.py:31-79`` collate: pad 0, attention mask), scores are the CLS
linear head.  Losses as ``asr_rescoring_amd/csrc/train.h`` (restated from the RescoreBERT
paper — **parity unpinned** against the reference's loss code).  No dropout.
"""
from __future__ import annotations

from typing import Dict, List, Sequence

import numpy as np
import torch

from .bert_ref import TorchBert


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
        self.opt = torch.optim.AdamW(list(self.model.w.values()), lr=lr, betas=betas, eps=eps,
                                     weight_decay=weight_decay)

    def scores(self, seqs: Sequence[Sequence[int]]) -> torch.Tensor:
        T = max(len(s) for s in seqs)
        ids = torch.zeros(len(seqs), T, dtype=torch.long)
        am = torch.zeros(len(seqs), T, dtype=torch.long)
        for i, s in enumerate(seqs):
            ids[i, :len(s)] = torch.as_tensor(list(s))
            am[i, :len(s)] = 1
        return self.model.cls_score(self.model.encoder(ids, am))

    @staticmethod
    def loss(sc, target, am, err, utt_off, kind: str, lam: float):
        t = torch.as_tensor(np.asarray(target, np.float32))
        md = ((sc - t) ** 2).mean()
        if kind == "MD":
            return md
        a = torch.as_tensor(np.asarray(am, np.float32))
        e = torch.as_tensor(np.asarray(err, np.float32))
        terms = []
        for u in range(len(utt_off) - 1):
            i0, i1 = int(utt_off[u]), int(utt_off[u + 1])
            c, eu = a[i0:i1] + sc[i0:i1], e[i0:i1]
            if kind == "MD_MWER":
                terms.append((torch.softmax(c, 0) * (eu - eu.mean())).sum())
            else:
                cs, es = float(c.detach().sum()), float(-eu.sum())
                tau = cs / es if es != 0.0 and cs / es > 0.0 else 1.0
                terms.append(-(torch.softmax(-eu, 0) * torch.log_softmax(c / tau, 0)).sum())
        return md + lam * torch.stack(terms).mean()

    def step(self, seqs, utt_off, target, am=None, err=None, kind="MD", lam=1.0, update=True):
        self.opt.zero_grad(set_to_none=False)
        sc = self.scores(seqs)
        loss = self.loss(sc, target, am, err, utt_off, kind, lam)
        loss.backward()
        if update:
            self.opt.step()
        return float(loss.detach()), sc.detach().numpy()

    def grad(self, key: str) -> np.ndarray:
        return self.model.w[key].grad.detach().numpy()

    def tensor(self, key: str) -> np.ndarray:
        return self.model.w[key].detach().numpy()


    def step_mlm(self, ids: np.ndarray, seq_off: np.ndarray, labels: np.ndarray, update=True) -> float:
        """BertForMaskedLM CE over every real position (pads ignored), mean; AdamW."""
        seqs = [ids[seq_off[i]:seq_off[i + 1]] for i in range(len(seq_off) - 1)]
        T = max(len(x) for x in seqs)
        x = torch.zeros(len(seqs), T, dtype=torch.long)
        am = torch.zeros(len(seqs), T, dtype=torch.long)
        lab = torch.full((len(seqs), T), -100, dtype=torch.long)
        for i, sq in enumerate(seqs):
            x[i, :len(sq)] = torch.as_tensor(sq.astype(np.int64))
            am[i, :len(sq)] = 1
            lab[i, :len(sq)] = torch.as_tensor(labels[seq_off[i]:seq_off[i + 1]].astype(np.int64))
        self.opt.zero_grad(set_to_none=False)
        logits = self.model.mlm_logits(self.model.encoder(x, am))
        loss = torch.nn.functional.cross_entropy(logits.view(-1, logits.shape[-1]), lab.view(-1), ignore_index=-100)
        loss.backward()
        if update:
            self.opt.step()
        return float(loss.detach())
