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
                 weight_decay=0.01):
        # own copies: TorchBert wraps numpy memory and AdamW updates in place
        self.model = TorchBert({k: np.array(v, np.float32, copy=True) for k, v in weights.items()
                                if not k.startswith("bert.pooler.") and not k.startswith("cls.")}, shape)
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
