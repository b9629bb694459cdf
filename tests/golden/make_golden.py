"""Generate the golden fixtures by running the REFERENCE code itself (this container only).

Run from the repo root:  ``python tests/golden/make_golden.py``  (needs /root/reference).

The reference is imported read-only from ``/root/reference`` with three stubs for packages
absent from this image: ``ruamel.yaml`` (used only by util/arg_parser.py),
``jiwer`` (bound to ``oracle.rescore_ref.corpus_cer`` — the jiwer boundary is therefore
"parity unpinned" except for the checks in tests/test_oracle_rescore.py) and
``bert_score`` (never called: the CER utility is used).  BERT comes from
``transformers`` (installed 5.15.0) with weights from ``asr_rescoring_amd.weights``.

Fixtures written (inputs + expected outputs only; no reference source):
  F1 pll_base.npz      3 utts x N=4 BERT-base MLM_PLL: per-row log p, per-hyp PLL
                       (MLM_PLL/main.py run_one_epoch + MLM_PLL/preprocess.py do_job)
  F2 cls_base.npz      RescoreBert scores for the same hypotheses (RescoreBert/model.py)
  F3 c1_plumbing.json  C1: 10 alfred test utts x N=10, synthesized hyps, real AM,
                       BERT-base PLL (F1 weights) via the reference run_one_epoch, then
                       rescore.rescore / get_highest_score_hyp over the 101-weight grid
  F4 rmbr.npz          RMBR mbr_decode (CER utility) for 5 utts x N=12, every k
  F5 pll_tiny.npz      tiny BERT (2 layers, H=256) PLL rows for fast kernel tests
  alfred_test_lengths.json  reference-length histogram (real-length synthetic variant)
"""
from __future__ import annotations

import importlib.util
import json
import os
import sys
import tempfile
import types

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, REPO)

from asr_rescoring_amd import data as D                      # noqa: E402
from asr_rescoring_amd.weights import (BERT_BASE, BERT_TINY,  # noqa: E402
                                       make_weights, weights_digest)
from oracle import rescore_ref                                # noqa: E402


def install_stubs():
    ry = types.ModuleType("ruamel.yaml")
    import yaml as _pyyaml
    ry.load = lambda f, Loader=None: _pyyaml.safe_load(f)
    ry.Loader = None
    ru = types.ModuleType("ruamel")
    ru.yaml = ry
    sys.modules["ruamel"] = ru
    sys.modules["ruamel.yaml"] = ry
    jw = types.ModuleType("jiwer")

    def cer(reference, hypothesis):
        if isinstance(reference, str):
            reference, hypothesis = [reference], [hypothesis]
        enc = lambda s: [ord(c) for c in s.strip()]          # noqa: E731
        return rescore_ref.corpus_cer([enc(r) for r in reference], [enc(h) for h in hypothesis])
    jw.cer = cer
    sys.modules["jiwer"] = jw
    bs = types.ModuleType("bert_score")
    bs.score = None
    sys.modules["bert_score"] = bs


def load_ref_module(name, relpath, extra_path=None):
    if extra_path:
        sys.path.insert(0, extra_path)
    spec = importlib.util.spec_from_file_location(name, os.path.join(REF, relpath))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


class IdTokenizer:
    """Feeds id strings through the reference's do_job: "345 678" -> ids."""

    def tokenize(self, s):
        return s.split()

    def convert_tokens_to_ids(self, toks):
        sp = {"[CLS]": D.CLS_ID, "[SEP]": D.SEP_ID, "[MASK]": D.MASK_ID}
        return [sp[t] if t in sp else int(t) for t in toks]


def hf_model(shape, weights, kind="mlm"):
    from transformers import BertConfig, BertForMaskedLM, BertModel
    cfg = BertConfig(vocab_size=shape.vocab, hidden_size=shape.hidden,
                     num_hidden_layers=shape.layers, num_attention_heads=shape.heads,
                     intermediate_size=shape.intermediate, max_position_embeddings=shape.max_pos,
                     layer_norm_eps=shape.ln_eps, hidden_act="gelu")
    m = BertForMaskedLM(cfg) if kind == "mlm" else BertModel(cfg)
    sd = {k: torch.from_numpy(v.copy()) for k, v in weights.items()
          if k in m.state_dict()}
    if kind != "mlm":
        sd = {k[len("bert."):]: v for k, v in ((k, torch.from_numpy(w.copy())) for k, w in weights.items())
              if k.startswith("bert.")}
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected
    assert all("position_ids" in k or "token_type_ids" in k for k in missing), missing
    return m.eval(), cfg


def reference_pll(main_mod, pre_mod, model, nb: D.NBest, per_row: bool):
    """Rows via the reference do_job, scores via the reference run_one_epoch (CPU)."""
    pre_mod.bert_tokenizer = IdTokenizer()
    rows = []
    for h in range(nb.n_hyp):
        words = " ".join(str(int(x)) for x in nb.hyp_words(h))
        rows = pre_mod.do_job(words, f"u{h}", f"h{h}", "for_scoring", rows)
    if per_row:
        for i, r in enumerate(rows):
            r["utt_id"], r["hyp_id"] = "rows", f"r{i}"
    out = {}
    for r in rows:
        out.setdefault(r["utt_id"], {})[r["hyp_id"]] = 0
    cfg = types.SimpleNamespace(device="cpu", batch_size=32, num_worker=0, shuffle=False)
    loader = main_mod.set_dataloader(cfg, main_mod.MyDataset(rows), for_scoring=True)
    res = main_mod.run_one_epoch(cfg, model, loader, output_score=out, train_mode=False, do_scoring=True)
    if per_row:
        return np.asarray([res["rows"][f"r{i}"] for i in range(len(rows))], np.float64), rows
    return np.asarray([res[f"u{h}"][f"h{h}"] for h in range(nb.n_hyp)], np.float64), rows


def short_nbest(n_utt, n_best, seed, vocab, lo, hi):
    return D.synthetic_nbest(n_utt, n_best, seed=seed, vocab=vocab, len_lo=lo, len_hi=hi)


def synthesize_hyps(ref: str, cers, rng, charset):
    out = []
    for c in cers:
        k = int(round(c * len(ref)))
        s = list(ref)
        pos = rng.choice(len(s), size=min(k, len(s)), replace=False)
        for p in pos:
            alt = s[p]
            while alt == s[p]:
                alt = charset[int(rng.integers(0, len(charset)))]
            s[p] = alt
        out.append("".join(s))
    return out


def main():
    install_stubs()
    torch.manual_seed(0)
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    main_mod = load_ref_module("ref_mlm_main", "MLM_PLL/main.py", REF)
    pre_mod = load_ref_module("ref_mlm_pre", "MLM_PLL/preprocess.py", REF)
    rb_mod = load_ref_module("ref_rb_model", "RescoreBert/model.py")
    rescore_mod = load_ref_module("ref_rescore", "rescore.py", REF)
    mbr_mod = load_ref_module("ref_mbr", "RMBR/mbr.py", os.path.join(REF, "RMBR"))
    uf_mod = sys.modules.get("utility_functions") or load_ref_module("utility_functions", "RMBR/utility_functions.py")

    # ---------------- F1: BERT-base PLL --------------------------------------------
    wb = make_weights(BERT_BASE, seed=1234, with_cls_linear=True, with_pooler=True)
    dig = weights_digest(wb)
    m, _ = hf_model(BERT_BASE, wb)
    nb = short_nbest(3, 4, seed=0, vocab=BERT_BASE.vocab, lo=3, hi=20)
    rows_lp, rows = reference_pll(main_mod, pre_mod, m, nb, per_row=True)
    pll, _ = reference_pll(main_mod, pre_mod, m, nb, per_row=False)
    np.savez(os.path.join(OUT, "pll_base.npz"), tokens=nb.tokens, hyp_off=nb.hyp_off,
             utt_off=nb.utt_off, row_lp=rows_lp, pll=pll,
             seed=1234, std=0.05, digest=np.array(dig))
    print("F1 rows", len(rows_lp), "pll", pll[:4])

    # ---------------- F2: RescoreBert --------------------------------------------------
    with tempfile.TemporaryDirectory() as td:
        bm, _ = hf_model(BERT_BASE, wb, kind="base")
        bm.save_pretrained(td)
        rb = rb_mod.RescoreBert(td).eval()
        with torch.no_grad():
            rb.linear.weight.copy_(torch.from_numpy(wb["linear.weight"]))
            rb.linear.bias.copy_(torch.from_numpy(wb["linear.bias"]))
            seqs = [torch.tensor(nb.tokens[nb.hyp_off[h]:nb.hyp_off[h + 1]], dtype=torch.long)
                    for h in range(nb.n_hyp)]
            from torch.nn.utils.rnn import pad_sequence
            ids = pad_sequence(seqs, batch_first=True)
            am = pad_sequence([torch.ones_like(s) for s in seqs], batch_first=True)
            cls = rb(ids, am).numpy().astype(np.float32)
    np.savez(os.path.join(OUT, "cls_base.npz"), tokens=nb.tokens, hyp_off=nb.hyp_off, cls=cls,
             digest=np.array(dig))
    print("F2 cls", cls[:4])
    del rb, bm

    # ---------------- F5: tiny BERT PLL ------------------------------------------------
    wt = make_weights(BERT_TINY, seed=7, with_cls_linear=True, with_pooler=True)
    mt, _ = hf_model(BERT_TINY, wt)
    nbt = short_nbest(6, 5, seed=3, vocab=BERT_TINY.vocab, lo=2, hi=40)
    rows_t, _ = reference_pll(main_mod, pre_mod, mt, nbt, per_row=True)
    pll_t, _ = reference_pll(main_mod, pre_mod, mt, nbt, per_row=False)
    with tempfile.TemporaryDirectory() as td:
        bmt, _ = hf_model(BERT_TINY, wt, kind="base")
        bmt.save_pretrained(td)
        rbt = rb_mod.RescoreBert(td).eval()
        with torch.no_grad():
            rbt.linear.weight.copy_(torch.from_numpy(wt["linear.weight"]))
            rbt.linear.bias.copy_(torch.from_numpy(wt["linear.bias"]))
            from torch.nn.utils.rnn import pad_sequence
            seqs = [torch.tensor(nbt.tokens[nbt.hyp_off[h]:nbt.hyp_off[h + 1]], dtype=torch.long)
                    for h in range(nbt.n_hyp)]
            cls_t = rbt(pad_sequence(seqs, batch_first=True),
                        pad_sequence([torch.ones_like(s) for s in seqs], batch_first=True)).numpy()
    np.savez(os.path.join(OUT, "pll_tiny.npz"), tokens=nbt.tokens, hyp_off=nbt.hyp_off,
             utt_off=nbt.utt_off, row_lp=rows_t, pll=pll_t, cls=cls_t.astype(np.float32),
             seed=7, digest=np.array(weights_digest(wt)))
    print("F5 rows", len(rows_t))

    # ---------------- F3: C1 plumbing (alfred test, 10 utts x N=10) --------------------
    base = os.path.join(REF, "espnet_data/alfred/test")
    ref_text = json.load(open(os.path.join(base, "ref_text.json"), encoding="utf-8"))
    hyps_score = json.load(open(os.path.join(base, "hyps_score.json"), encoding="utf-8"))
    hyps_cer = json.load(open(os.path.join(base, "hyps_cer.json"), encoding="utf-8"))
    lengths = [len(v) for v in ref_text.values()]
    hist = np.bincount(lengths).tolist()
    json.dump({"source": "espnet_data/alfred/test/ref_text.json", "length_counts": hist},
              open(os.path.join(OUT, "alfred_test_lengths.json"), "w"))
    uids = list(ref_text)[:10]
    charset = sorted(set("".join(ref_text.values())))
    rng = np.random.Generator(np.random.PCG64(0))
    hyps_text = {u: dict(zip(hyps_cer[u], synthesize_hyps(ref_text[u], list(hyps_cer[u].values()),
                                                          rng, charset))) for u in uids}
    tok = D.CharTokenizer(charset)
    words = [[tok.encode_words(t) for t in hyps_text[u].values()] for u in uids]
    am = [list(hyps_score[u].values()) for u in uids]
    nb1 = D.from_lists(words, am, [tok.encode_words(ref_text[u]) for u in uids], uids)
    # C1 = bert-base-chinese shape (V=21128 covers the char ids), the F1 weights
    assert 106 + len(charset) <= BERT_BASE.vocab
    shape_c1 = BERT_BASE
    mc, _ = hf_model(shape_c1, wb)
    lm, _ = reference_pll(main_mod, pre_mod, mc, nb1, per_row=False)
    lm_json = D.scores_to_json_dict(nb1, lm)
    am_l = rescore_mod.dict_to_list({u: hyps_score[u] for u in uids})
    lm_l = rescore_mod.dict_to_list(lm_json)
    hy_l = rescore_mod.dict_to_list(hyps_text)
    ref_l = rescore_mod.dict_to_list({u: ref_text[u] for u in uids})
    cfg = types.SimpleNamespace(n_best=10)
    best_w, best_cer = rescore_mod.find_best_weight(am_l, lm_l, hy_l, ref_l, cfg)
    hyps_len = [[len(h) for h in utt[:10]] for utt in hy_l]
    argmaxes, cers = [], []
    for w in np.arange(0.0, 1.01, 0.01):
        fs = rescore_mod.rescore(w, hyps_len, am_l, lm_l, cfg)
        argmaxes.append(np.argmax(fs, axis=-1).tolist())
        cers.append(sys.modules["jiwer"].cer(ref_l, rescore_mod.get_highest_score_hyp(fs, hy_l)))
    json.dump({"utt_ids": uids, "ref_text": {u: ref_text[u] for u in uids},
               "hyps_text": hyps_text, "hyps_score": {u: hyps_score[u] for u in uids},
               "hyps_cer": {u: hyps_cer[u] for u in uids}, "charset": "".join(charset),
               "model_seed": 1234, "model_vocab": shape_c1.vocab, "lm": lm_json,
               "argmax_per_weight": argmaxes, "cer_per_weight": cers,
               "best_weight": float(best_w), "best_cer": float(best_cer)},
              open(os.path.join(OUT, "c1_plumbing.json"), "w", encoding="utf-8"),
              ensure_ascii=False, indent=1)
    print("F3 best_w", best_w, "cer", best_cer)

    # ---------------- F4: RMBR CER utility ---------------------------------------------
    nb4 = D.synthetic_nbest(5, 12, seed=4, vocab=200, len_lo=3, len_hi=12, max_edits=3)
    hyps4 = [[" ".join(chr(0x4e00 + int(x)) for x in nb4.hyp_words(h)).replace(" ", "")
              for h in range(nb4.utt_off[u], nb4.utt_off[u + 1])] for u in range(nb4.n_utt)]
    util = uf_mod.CerScoreFunction(None)
    per_k = {}
    for k in range(2, 13):
        pred, scores = mbr_mod.mbr_decode(k, hyps4, util)
        per_k[str(k)] = {"argmax": [h.index(p) for h, p in zip(hyps4, pred)],
                         "scores": scores.numpy().astype(np.float32).tolist()}
    np.savez(os.path.join(OUT, "rmbr.npz"), tokens=nb4.tokens, hyp_off=nb4.hyp_off,
             utt_off=nb4.utt_off, **{f"argmax_k{k}": np.asarray(v["argmax"], np.int64) for k, v in per_k.items()},
             **{f"scores_k{k}": np.asarray(v["scores"], np.float32) for k, v in per_k.items()})
    print("F4 done")


if __name__ == "__main__":
    main()
