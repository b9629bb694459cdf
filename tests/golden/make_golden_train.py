"""Training fixtures made by running the REFERENCE training code itself (this container only).

Run from the repo root:  ``python tests/golden/make_golden_train.py``  (needs /root/reference).

The reference modules are imported read-only with the stubs of ``make_golden.py``
(``ruamel.yaml``, ``jiwer``, ``bert_score``).  BERT comes from ``transformers`` with weights
from ``asr_rescoring_amd.weights`` (BERT_TINY shape).  Dropout is switched off through the
model CONFIG (``hidden_dropout_prob = attention_probs_dropout_prob = 0``) — the reference
code runs unchanged, but its ``model.train()`` then adds no noise, so the training step is
deterministic and reproducible by another implementation.  Batches are built by the
reference's own ``collate`` / ``set_dataloader`` (shuffle False, as its train configs).

Fixtures written (inputs + expected outputs only; no reference source):
  F6 train_rb_{MD,MD_MWER,MD_MWED}.npz
     RescoreBert/main.py:82-163 run_one_epoch(grad_update=True, train=True) for 2 epochs
     (AdamW re-created per epoch, lr 1e-3, md_loss_weight 0.05, batch_size 2 utterances x
     n_best 3) on 4 train utterances, the dev loss after each epoch (grad_update=False,
     train=True), the dev CLS scores after training (train=False), and every parameter's
     update as a sketch (sum, L2 norm, dot with a seeded Gaussian probe; the whole update for
     tensors of <= 1024 elements).
  F7 train_mlm.npz
     MLM_PLL/main.py:73-114 run_one_epoch(train_mode=True) for 2 epochs on do_job rows
     (MLM_PLL/preprocess.py:9-30) of 3 sentences, batch 4 rows (pad_sequence: labels padded
     with 0, CE over all B*T positions), dev loss per epoch, the same update sketches.
"""
from __future__ import annotations

import os
import sys
import tempfile
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as G                                       # noqa: E402

from asr_rescoring_amd import data as D                      # noqa: E402
from asr_rescoring_amd.weights import BERT_TINY, make_weights, weights_digest  # noqa: E402

REF = G.REF
OUT = G.OUT
SEED_W = 11


def sketch(before: dict, after: dict, prefix: str = "") -> dict:
    """Per tensor: (sum, L2 norm, probe dot) of the update, probe = N(0,1) from PCG64(i)."""
    out = {}
    for i, k in enumerate(sorted(before)):
        d = (after[k].astype(np.float64) - before[k].astype(np.float64)).ravel()
        r = np.random.Generator(np.random.PCG64(1000 + i)).standard_normal(d.size)
        out[f"{prefix}sk/{k}"] = np.asarray([d.sum(), np.linalg.norm(d), float(d @ r)], np.float64)
        if d.size <= 1024:
            out[f"{prefix}full/{k}"] = d.astype(np.float32)
    return out


def no_dropout_cfg(shape):
    from transformers import BertConfig
    return BertConfig(vocab_size=shape.vocab, hidden_size=shape.hidden, num_hidden_layers=shape.layers,
                      num_attention_heads=shape.heads, intermediate_size=shape.intermediate,
                      max_position_embeddings=shape.max_pos, layer_norm_eps=shape.ln_eps, hidden_act="gelu",
                      hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)


def rb_rows(nb, pll, cer, keys):
    rows = []
    for h in range(nb.n_hyp):
        t = nb.tokens[nb.hyp_off[h]:nb.hyp_off[h + 1]].tolist()
        u, hid = keys[h]
        rows.append({"utt_id": u, "hyp_id": hid, "hyps_token_ids": t, "attention_masks": [1] * len(t),
                     "mlm_pll_score": float(pll[h]), "hyps_am_score": float(nb.am[h]), "hyps_cer": float(cer[h])})
    return rows


def rb_data(seed, n_utt, n_best):
    nb = D.synthetic_nbest(n_utt, n_best, seed=seed, vocab=BERT_TINY.vocab, len_lo=2, len_hi=14)
    rng = np.random.default_rng(seed)
    pll = rng.normal(-1.0, 1.0, nb.n_hyp)   # teacher scores near the student's, so MD does not drown MWER / MWED
    # CER values of the reference's domain: k / len(ref)
    cer = rng.integers(0, 4, nb.n_hyp) / rng.integers(5, 15, nb.n_hyp)
    keys = [(f"u{u}", f"hyp_{h - nb.utt_off[u] + 1}") for u in range(nb.n_utt)
            for h in range(nb.utt_off[u], nb.utt_off[u + 1])]
    return nb, pll, cer, keys


def rescorebert_fixtures(main_rb, rb_mod):
    from transformers import BertModel
    w = make_weights(BERT_TINY, seed=SEED_W, with_cls_linear=True, with_pooler=True)
    tr_nb, tr_pll, tr_cer, tr_keys = rb_data(21, 4, 3)
    dv_nb, dv_pll, dv_cer, dv_keys = rb_data(22, 2, 3)
    for method in ("MD", "MD_MWER", "MD_MWED"):
        torch.manual_seed(0)
        with tempfile.TemporaryDirectory() as td:
            bm = BertModel(no_dropout_cfg(BERT_TINY))
            sd = {k[len("bert."):]: torch.from_numpy(v.copy()) for k, v in w.items() if k.startswith("bert.")}
            missing, unexpected = bm.load_state_dict(sd, strict=False)
            assert not unexpected and all("position_ids" in k or "token_type_ids" in k for k in missing), missing
            bm.save_pretrained(td)
            model = rb_mod.RescoreBert(td)
        with torch.no_grad():
            model.linear.weight.copy_(torch.from_numpy(w["linear.weight"]))
            model.linear.bias.copy_(torch.from_numpy(w["linear.bias"]))
        before = {k: v.detach().numpy().copy() for k, v in model.state_dict().items()}
        cfg = types.SimpleNamespace(task="training", method=method, n_best=3, batch_size=2, md_loss_weight=0.05,
                                    lr=1e-3, device="cpu", dataloader=types.SimpleNamespace(num_worker=0))
        tr_loader = main_rb.set_dataloader(cfg, main_rb.MyDataset(rb_rows(tr_nb, tr_pll, tr_cer, tr_keys)),
                                           shuffle=False)
        dv_rows = rb_rows(dv_nb, dv_pll, dv_cer, dv_keys)
        dv_loader = main_rb.set_dataloader(cfg, main_rb.MyDataset(dv_rows), shuffle=False)
        tl, dl = [], []
        for _ in range(2):
            tl.append(main_rb.run_one_epoch(cfg, model, tr_loader, grad_update=True, train=True))
            dl.append(main_rb.run_one_epoch(cfg, model, dv_loader, grad_update=False, train=True))
        fmt = {}
        for u, h in dv_keys:
            fmt.setdefault(u, {})[h] = 0
        with torch.no_grad():
            sc = main_rb.run_one_epoch(cfg, model, dv_loader, output_score=fmt, grad_update=False, train=False)
        dev_scores = np.asarray([sc[u][h] for u, h in dv_keys], np.float32)
        after = {k: v.detach().numpy() for k, v in model.state_dict().items()}
        np.savez(os.path.join(OUT, f"train_rb_{method}.npz"),
                 tr_tokens=tr_nb.tokens, tr_hyp_off=tr_nb.hyp_off, tr_utt_off=tr_nb.utt_off,
                 tr_pll=tr_pll.astype(np.float32), tr_am=tr_nb.am.astype(np.float32), tr_cer=tr_cer.astype(np.float32),
                 dv_tokens=dv_nb.tokens, dv_hyp_off=dv_nb.hyp_off, dv_utt_off=dv_nb.utt_off,
                 dv_pll=dv_pll.astype(np.float32), dv_am=dv_nb.am.astype(np.float32), dv_cer=dv_cer.astype(np.float32),
                 train_loss=np.asarray(tl, np.float64), dev_loss=np.asarray(dl, np.float64), dev_scores=dev_scores,
                 n_best=3, batch_size=2, md_loss_weight=0.05, lr=1e-3, weight_seed=SEED_W,
                 digest=np.array(weights_digest(w)), **sketch(before, after))
        print(method, "train", tl, "dev", dl)


def mlm_fixture(main_mlm, pre_mod):
    from transformers import BertForMaskedLM
    w = make_weights(BERT_TINY, seed=SEED_W + 1)
    torch.manual_seed(0)
    m = BertForMaskedLM(no_dropout_cfg(BERT_TINY))
    sd = {k: torch.from_numpy(v.copy()) for k, v in w.items() if k in m.state_dict()}
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert not unexpected and all("position_ids" in k or "token_type_ids" in k for k in missing), missing
    pre_mod.bert_tokenizer = G.IdTokenizer()

    def rows_of(seed, n):
        nb = D.synthetic_nbest(n, 1, seed=seed, vocab=BERT_TINY.vocab, len_lo=2, len_hi=7)
        rows = []
        for h in range(nb.n_hyp):
            rows = pre_mod.do_job(" ".join(str(int(x)) for x in nb.hyp_words(h)), f"u{h}", None, "for_training", rows)
        return rows
    tr_rows, dv_rows = rows_of(31, 3), rows_of(32, 2)
    before = {k: v.detach().numpy().copy() for k, v in m.state_dict().items() if not k.startswith("cls.predictions.decoder.")}
    cfg = types.SimpleNamespace(device="cpu", lr=1e-3, batch_size=4, num_worker=0, shuffle=False)
    tr_loader = main_mlm.set_dataloader(cfg, tr_rows, False)
    dv_loader = main_mlm.set_dataloader(cfg, dv_rows, True)
    tl, dl = [], []
    for _ in range(2):
        tl.append(main_mlm.run_one_epoch(cfg, m, tr_loader, output_score=None, train_mode=True, do_scoring=False))
        with torch.no_grad():
            dl.append(main_mlm.run_one_epoch(cfg, m, dv_loader, output_score=None, train_mode=False, do_scoring=False))
    after = {k: v.detach().numpy() for k, v in m.state_dict().items() if not k.startswith("cls.predictions.decoder.")}

    def flat(rows, key):
        return np.asarray([x for r in rows for x in r[key]], np.int32)
    off = lambda rows: np.concatenate([[0], np.cumsum([len(r["input_ids"]) for r in rows])]).astype(np.int32)  # noqa: E731
    np.savez(os.path.join(OUT, "train_mlm.npz"),
             tr_ids=flat(tr_rows, "input_ids"), tr_labels=flat(tr_rows, "labels"), tr_off=off(tr_rows),
             dv_ids=flat(dv_rows, "input_ids"), dv_labels=flat(dv_rows, "labels"), dv_off=off(dv_rows),
             train_loss=np.asarray(tl, np.float64), dev_loss=np.asarray(dl, np.float64),
             batch_size=4, lr=1e-3, weight_seed=SEED_W + 1, digest=np.array(weights_digest(w)), **sketch(before, after))
    print("MLM train", tl, "dev", dl)


def main():
    G.install_stubs()
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    main_mlm = G.load_ref_module("ref_mlm_main", "MLM_PLL/main.py", REF)
    pre_mod = G.load_ref_module("ref_mlm_pre", "MLM_PLL/preprocess.py", REF)
    sys.path.insert(0, os.path.join(REF, "RescoreBert"))
    rb_mod = G.load_ref_module("model", "RescoreBert/model.py")
    sys.modules["model"] = rb_mod
    main_rb = G.load_ref_module("ref_rb_main", "RescoreBert/main.py", REF)
    rescorebert_fixtures(main_rb, rb_mod)
    mlm_fixture(main_mlm, pre_mod)


if __name__ == "__main__":
    main()
