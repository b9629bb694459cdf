"""ORACLE (test infrastructure only) — PyTorch-CPU fp32 restatement of the reference scorers.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker / the timed CPU baseline.  The product path
(``asr_rescoring_amd``) never imports it.

What is restated (no ``transformers`` import; BERT math written out with torch ops):

* ``MLM_PLL/preprocess.py:9-30`` ``do_job``: L masked copies per hypothesis,
  ``input_ids = [CLS] + w[:p] + [MASK] + w[p+1:] + [SEP]``, ``mask_pos = p + 1``,
  ``labels = [CLS] + w + [SEP]``.
* ``MLM_PLL/main.py:28-54`` ``collate`` (``pad_sequence`` with 0) and batches of
  ``dataloader.batch_size`` = 32 rows in order (``MLM_PLL/config/score.yaml:16``, no shuffle).
* ``MLM_PLL/main.py:89-109``: ``BertForMaskedLM`` forward with ``labels`` (logits at every
  position + CrossEntropy over all positions — the reference's work pattern, kept for the
  CPU baseline), ``log_softmax(logits[i, mask_pos_i])[labels[i, mask_pos_i]]``, Python
  float64 ``+=`` per hypothesis in row order (``:105-107``).
* transformers ``modeling_bert.py`` (v5.15.0 installed; the reference pins none):
  ``BertEmbeddings`` :53-108 (word + token_type[0] + position, LayerNorm eps 1e-12),
  ``eager_attention_forward`` :111-136 (scale head_dim**-0.5, additive pad mask, softmax),
  ``BertSelfOutput`` :282-293, ``BertIntermediate`` :325-337 (erf GELU),
  ``BertOutput`` :340-351, ``BertPredictionHeadTransform`` :466-480,
  ``BertLMPredictionHead`` :483-496 (decoder tied to word embeddings).
* ``RescoreBert/model.py:13-21``: ``BertModel`` (pooler computed, unused) → CLS hidden →
  ``Linear(768, 1)`` → squeeze; batches of ``batch_size * n_best`` rows
  (``RescoreBert/main.py:75``), ``.item()`` per hypothesis (``:157-158``).

Pinned against the reference itself: ``tests/golden/make_golden.py`` runs the imported
reference (``MLM_PLL.main.run_one_epoch``, ``RescoreBert.model.RescoreBert``) on the same
seeded weights and inputs; ``tests/test_oracle_golden.py`` checks this module against it.
"""
from __future__ import annotations


import os
from typing import Dict, List, Tuple

import numpy as np
import torch
import torch.nn.functional as Fn


class TorchBert:
    """fp32 BERT from an HF-keyed weight dict (numpy arrays); on the CPU (the oracle), or on a
    GPU as the plain torch fp32 reference of a larger parity test (``device="cuda"``)."""

    def __init__(self, weights: Dict[str, np.ndarray], shape, device: str = "cpu"):
        self.s = shape
        self.w = {k: torch.from_numpy(np.ascontiguousarray(v)).to(device) for k, v in weights.items()}
        self.device = device

    def _lin(self, x, key):
        return Fn.linear(x, self.w[key + ".weight"], self.w[key + ".bias"])

    def _ln(self, x, key):
        return Fn.layer_norm(x, (self.s.hidden,), self.w[key + ".weight"], self.w[key + ".bias"],
                             eps=self.s.ln_eps)

    def encoder(self, input_ids: torch.Tensor, attention_mask: torch.Tensor,
                last_layer_rows: torch.Tensor | None = None, drop: dict | None = None) -> torch.Tensor:
        """input_ids/attention_mask int64 [B, T] → last hidden [B, T, H] (modeling_bert.py:53-351).

        ``drop`` (training with dropout): multipliers (0 or 1/(1-p)) at the places BERT's train
        mode applies nn.Dropout — "emb" [B, T, H] after the embedding LayerNorm; per layer i
        ("attn", i) [B, heads, T, T] on the attention probabilities, ("so", i) / ("out", i)
        [B, T, H] on the BertSelfOutput / BertOutput dense outputs before the residual add."""
        s = self.s
        B, T = input_ids.shape
        pos = torch.arange(T, device=self.device)
        e = "bert.embeddings."
        # nn.Embedding(padding_idx=pad_token_id) (modeling_bert BertEmbeddings): the lookup of
        # the pad id passes no gradient to its row (the tied decoder still does)
        x = (Fn.embedding(input_ids, self.w[e + "word_embeddings.weight"], padding_idx=s.pad_id)
             + self.w[e + "token_type_embeddings.weight"][0]
             + self.w[e + "position_embeddings.weight"][pos][None])
        x = self._ln(x, e + "LayerNorm")
        if drop is not None:
            x = x * drop["emb"]
        # additive mask: 0 keep, finfo.min drop (transformers bidirectional mask semantics)
        add = (1.0 - attention_mask[:, None, None, :].to(x.dtype)) * torch.finfo(x.dtype).min
        nh, hd = s.heads, s.head_dim
        for i in range(s.layers):
            p = f"bert.encoder.layer.{i}."
            q = self._lin(x, p + "attention.self.query").view(B, T, nh, hd).transpose(1, 2)
            k = self._lin(x, p + "attention.self.key").view(B, T, nh, hd).transpose(1, 2)
            v = self._lin(x, p + "attention.self.value").view(B, T, nh, hd).transpose(1, 2)
            sc = torch.matmul(q, k.transpose(2, 3)) * (hd ** -0.5) + add
            pr = torch.softmax(sc, dim=-1)
            if drop is not None:
                pr = pr * drop[("attn", i)]
            ctx = torch.matmul(pr, v).transpose(1, 2).reshape(B, T, s.hidden)
            so = self._lin(ctx, p + "attention.output.dense")
            if drop is not None:
                so = so * drop[("so", i)]
            x = self._ln(so + x, p + "attention.output.LayerNorm")
            it = Fn.gelu(self._lin(x, p + "intermediate.dense"))
            out = self._lin(it, p + "output.dense")
            if drop is not None:
                out = out * drop[("out", i)]
            x = self._ln(out + x, p + "output.LayerNorm")
        return x

    def mlm_logits(self, hidden: torch.Tensor) -> torch.Tensor:
        """BertOnlyMLMHead (modeling_bert.py:466-506): transform + tied decoder + bias."""
        c = "cls.predictions."
        t = self._ln(Fn.gelu(self._lin(hidden, c + "transform.dense")), c + "transform.LayerNorm")
        return Fn.linear(t, self.w["bert.embeddings.word_embeddings.weight"], self.w[c + "bias"])

    def cls_score(self, hidden: torch.Tensor) -> torch.Tensor:
        """RescoreBert/model.py:19-20 — CLS hidden → Linear(H, 1) → squeeze."""
        return Fn.linear(hidden[:, 0, :], self.w["linear.weight"], self.w["linear.bias"]).squeeze(-1)

    def pooler(self, hidden: torch.Tensor) -> torch.Tensor:
        """BertPooler (modeling_bert.py:451-462): computed by RescoreBert, never used."""
        return torch.tanh(self._lin(hidden[:, 0], "bert.pooler.dense"))


# ---------------------------------------------------------------------------------------
# Reference work patterns
# ---------------------------------------------------------------------------------------

def pll_rows(tokens: np.ndarray, hyp_off: np.ndarray, mask_id: int = 103):
    """``do_job`` (MLM_PLL/preprocess.py:11-28) over every hypothesis, in row order.

    Yields (hyp_index, input_ids list, mask_pos, labels list)."""
    for h in range(len(hyp_off) - 1):
        seq = [int(x) for x in tokens[hyp_off[h]:hyp_off[h + 1]]]
        L = len(seq) - 2
        for p in range(L):
            ids = list(seq)
            ids[p + 1] = mask_id
            yield h, ids, p + 1, seq


def _pad(rows: List[List[int]]) -> torch.Tensor:
    T = max(len(r) for r in rows)
    out = torch.zeros(len(rows), T, dtype=torch.long)
    for i, r in enumerate(rows):
        out[i, :len(r)] = torch.tensor(r, dtype=torch.long)
    return out


def pll_reference_pattern(model: TorchBert, tokens: np.ndarray, hyp_off: np.ndarray,
                          batch_size: int = 32, full_head: bool = True
                          ) -> Tuple[np.ndarray, np.ndarray]:
    """MLM_PLL scoring exactly as ``run_one_epoch(do_scoring=True)`` (MLM_PLL/main.py:73-114).

    Returns (row_logprob float32 [R], pll float64 [H]).  ``full_head`` keeps the
    reference's all-position logits + CE loss (the CPU-baseline work pattern); False
    computes the head only at the masked rows (same values, faster checker).
    """
    n_hyp = len(hyp_off) - 1
    pll = [0.0] * n_hyp                      # Python float64 accumulation (:106-107)
    row_lp: List[float] = []
    rows = list(pll_rows(tokens, hyp_off, model.s.mask_id))
    with torch.no_grad():
        for b0 in range(0, len(rows), batch_size):
            chunk = rows[b0:b0 + batch_size]
            ids = _pad([r[1] for r in chunk]).to(model.device)
            am = _pad([[1] * len(r[1]) for r in chunk]).to(model.device)
            labels = _pad([r[3] for r in chunk]).to(model.device)
            mpos = [r[2] for r in chunk]
            hid = model.encoder(ids, am)
            rng = list(range(len(chunk)))
            if full_head:
                logits = model.mlm_logits(hid)
                _loss = Fn.cross_entropy(logits.view(-1, logits.shape[-1]), labels.view(-1))
                tok_logits = logits[rng, mpos, :]
            else:
                tok_logits = model.mlm_logits(hid[rng, mpos, :])
            lsm = tok_logits.log_softmax(dim=-1)
            lab = labels[rng, mpos]
            sc = lsm[rng, lab].tolist()
            for r, s in zip(chunk, sc):
                pll[r[0]] += s
                row_lp.append(s)
    return np.asarray(row_lp, np.float32), np.asarray(pll, np.float64)


def masked_logprob_ref(model: TorchBert, input_ids: np.ndarray, attention_mask: np.ndarray,
                       labels: np.ndarray, mask_pos: np.ndarray) -> np.ndarray:
    """``token_score`` of MLM_PLL/main.py:101-105 for one padded batch."""
    with torch.no_grad():
        ids = torch.from_numpy(input_ids.astype(np.int64))
        am = torch.from_numpy(attention_mask.astype(np.int64))
        hid = model.encoder(ids, am)
        rng = list(range(ids.shape[0]))
        mp = [int(x) for x in mask_pos]
        lsm = model.mlm_logits(hid[rng, mp, :]).log_softmax(dim=-1)
        lab = torch.from_numpy(labels.astype(np.int64))[rng, mp]
        return lsm[rng, lab].numpy().astype(np.float32)


def cls_reference_pattern(model: TorchBert, tokens: np.ndarray, hyp_off: np.ndarray,
                          batch_rows: int = 150, with_pooler: bool = False) -> np.ndarray:
    """RescoreBert scoring (RescoreBert/main.py:82-102,156-158): fp32 per hypothesis."""
    out: List[float] = []
    n_hyp = len(hyp_off) - 1
    with torch.no_grad():
        for h0 in range(0, n_hyp, batch_rows):
            hs = range(h0, min(n_hyp, h0 + batch_rows))
            seqs = [[int(x) for x in tokens[hyp_off[h]:hyp_off[h + 1]]] for h in hs]
            ids = _pad(seqs)
            am = _pad([[1] * len(s) for s in seqs])
            hid = model.encoder(ids, am)
            if with_pooler:
                model.pooler(hid)
            out.extend(float(x) for x in model.cls_score(hid))   # .item() per hyp
    return np.asarray(out, np.float32)


def set_cpu_threads() -> int:
    n = len(os.sched_getaffinity(0))
    n = min(n, int(os.environ.get("OMP_NUM_THREADS", n)))
    torch.set_num_threads(max(1, n))
    return torch.get_num_threads()


def forward_flops(T: int, shape) -> float:
    """Canonical algorithmic FLOPs of one MLM_PLL forward."""
    H, F, V, nl = shape.hidden, shape.intermediate, shape.vocab, shape.layers
    dense = 2 * (4 * H * H + 2 * H * F)
    enc = (nl - 1) * (T * dense + 4 * T * T * H)
    last = 4 * T * H * H + (2 * H * H + 4 * T * H + 2 * H * H + 4 * H * F)
    head = 2 * (H * H + H * V)
    return float(enc + last + head)



