"""Command-line drivers with the reference's entry points, YAML keys and output files.

  python -m asr_rescoring_amd.cli mlm_pll     --config score.yaml    # MLM_PLL/main.py (task: scoring)
  python -m asr_rescoring_amd.cli mlm_finetune --config train.yaml   # MLM_PLL/main.py (task: train)
  python -m asr_rescoring_amd.cli rescorebert --config MD_score.yaml # RescoreBert/main.py (task: scoring)
  python -m asr_rescoring_amd.cli rescorebert_train --config MD.yaml # RescoreBert/main.py (task: train)
  python -m asr_rescoring_amd.cli rescore     --config rescore.yaml  # rescore.py
  python -m asr_rescoring_amd.cli rmbr        --config CER.yaml      # RMBR/main.py (utility: cer / bertscore)

Differences forced by the offline image (no model hub): ``model.bert`` cannot be fetched,
so weights come from ``checkpoint_path`` (an HF-keyed state_dict, loaded with
``torch.load(weights_only=True)`` or safetensors) or, for testing, from the seeded
generator when ``random_init_seed`` is set.  The tokenizer is ``BertTokenizer``-like
per-character for CJK (``data.CharTokenizer``) built from the data, unless ``model.vocab``
names a ``vocab.txt`` — then the native BertTokenizer-compatible ``frontend.NativeTokenizer``
(and score JSON is written by the native ``frontend.json_saving``).  Extra keys: ``precision`` (fp16 / fp16x3), ``max_rows``,
``mode`` (rescore fusion formula: norm / legacy / am_norm).
"""
from __future__ import annotations

import json
import logging
import os
import sys
from typing import Dict, List

import numpy as np

from . import data as D
from .config import ArgParser, get
from .weights import BERT_BASE, load_state_dict_file, make_weights


def json_saving(path, data):
    """util/saving.py:14-16; native writer (frontend.json_saving) for score files."""
    from .frontend import json_saving as native
    native(path, data)


def _load(path):
    return json.load(open(path, "r", encoding="utf-8"))


def _weights(cfg, kind: str):
    ck = get(cfg, "checkpoint_path")
    if ck and os.path.exists(ck):
        return load_state_dict_file(ck)   # HF keys (bert.* [+ linear.* for RescoreBert])
    seed = get(cfg, "random_init_seed")
    if seed is None:
        raise FileNotFoundError(f"checkpoint_path {ck!r} not found (set random_init_seed to score with "
                                "seeded random weights)")
    return make_weights(BERT_BASE, seed=int(seed), with_cls_linear=(kind == "cls"), with_pooler=(kind == "cls"))


def _tokenizer(cfg, texts: List[str]):
    v = get(cfg, "model.vocab")
    if v and os.path.exists(v):
        from .frontend import NativeTokenizer          # BertTokenizer-compatible, native
        return NativeTokenizer(v)
    chars = sorted({c for t in texts for c in t})
    return D.CharTokenizer(chars)


def _nbest_tokens(hyps_text: Dict[str, Dict[str, str]], tok, max_utt=1 << 30, n_best=1 << 30):
    words, keys = [], []
    for u, (uid, hyps) in enumerate(hyps_text.items()):
        if u == max_utt:
            break
        row = []
        for k, (hid, text) in enumerate(hyps.items()):
            if k == n_best:
                break
            row.append(tok.encode_words(text))
            keys.append((uid, hid))
        words.append(row)
    return D.from_lists(words), keys


# --------------------------------------------------------------------------------------
def mlm_pll(cfg) -> Dict[str, str]:
    """MLM_PLL/main.py:164-203 (pll_bert_scoring).  Accepts the reference's preprocessed
    rows (``*_data_path``: do_job output) or raw ``*_hyps_text_path`` JSON.

    Launched with torchrun (WORLD_SIZE > 1): one process per GPU, each scores a contiguous,
    cost-balanced utterance range (``shard.plan_shards``); the scores meet in one all-gather
    (RCCL) and rank 0 writes the JSON (the reference is single-process)."""
    from . import shard
    from .scorer import PLLScorer
    rank, world, local = shard.init_from_env()
    device = local if world > 1 else _dev(cfg)
    scorer = PLLScorer(_weights(cfg, "mlm"), BERT_BASE, device=device, max_rows=get(cfg, "max_rows", 65536),
                       precision=get(cfg, "precision", "fp16x3"))
    out_files = {}
    for split in ("train", "dev", "test"):
        rows_path = get(cfg, f"{split}_data_path")
        text_path = get(cfg, f"{split}_hyps_text_path")
        if rows_path and os.path.exists(rows_path):
            rows = _load(rows_path)[:get(cfg, "num_of_data", 1 << 62)]
            output_score = _score_rows_sharded(scorer, rows, rank, world)
        elif text_path and os.path.exists(text_path):
            hyps = _load(text_path)
            tok = _tokenizer(cfg, [t for h in hyps.values() for t in h.values()])
            nb, keys = _nbest_tokens(hyps, tok)
            both = shard.score_sharded(nb, lambda sub: scorer.score_nbest(sub.tokens, sub.hyp_off))
            pll = both[1].cpu().numpy()
            output_score = {}
            for (u, h), s in zip(keys, pll):
                output_score.setdefault(u, {})[h] = float(s)
        else:
            continue
        path = cfg.output_path + f"{split}_lm.json"          # MLM_PLL/main.py:203 naming
        if rank == 0:
            json_saving(path, output_score)
        out_files[split] = path
    scorer.close()
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    return out_files


def _score_rows_sharded(scorer, rows, rank: int, world: int) -> Dict[str, Dict[str, float]]:
    """do_job rows (MLM_PLL/preprocess.py:9-30) scored by ``PLLScorer.run_one_epoch``; with
    several ranks each takes a contiguous, cost-balanced run of whole utterances and the
    per-row log-probs are exchanged once; every rank then forms ``output_score`` in the
    reference's row order (MLM_PLL/main.py:106-107)."""
    from . import shard
    output_score: Dict[str, Dict[str, float]] = {}
    for r in rows:                                       # MLM_PLL/main.py:189-193
        if r["hyp_id"] == "hyp_1":
            output_score[r["utt_id"]] = {}
        output_score[r["utt_id"]][r["hyp_id"]] = 0
    import torch
    import torch.distributed as dist
    if world == 1 and not dist.is_initialized():
        allv = scorer.row_logprobs(rows).cpu().tolist() if rows else []
        for r, s in zip(rows, allv):
            output_score[r["utt_id"]][r["hyp_id"]] += s
        return output_score
    # utterance runs of consecutive rows; cost = token rows
    starts = [i for i, r in enumerate(rows) if i == 0 or r["utt_id"] != rows[i - 1]["utt_id"]] + [len(rows)]
    costs = [sum(len(rows[i]["input_ids"]) for i in range(a, b)) for a, b in zip(starts, starts[1:])]
    parts = shard.plan_shards(costs, world)
    bounds = [(starts[a], starts[b]) for a, b in parts]
    r0, r1 = bounds[rank]
    lp = scorer.row_logprobs(rows[r0:r1]) if r1 > r0 else torch.zeros(0, device=scorer.device)
    counts = [b - a for a, b in bounds]
    dev = torch.device("cpu") if dist.get_backend() == "gloo" else scorer.device
    allv = shard.gather_scores(lp.to(dev, torch.float32)[None], counts)[0].cpu().tolist()
    for r, s in zip(rows, allv):
        output_score[r["utt_id"]][r["hyp_id"]] += s
    return output_score


def _save_checkpoint(output_path: str, state: Dict[str, np.ndarray], n: int) -> str:
    """util/saving.py:7-11 model_saving: ``checkpoint_{n}.pth`` (torch.save of the HF-keyed
    state_dict; loadable with ``torch.load(weights_only=True)`` as ``checkpoint_path``)."""
    import torch
    path = os.path.join(output_path, f"checkpoint_{n}.pth")
    torch.save({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in state.items()}, path)
    return path


def _dropout_args(cfg) -> Dict[str, float]:
    """BERT train-mode dropout of the trainers: BertConfig's defaults (hidden_dropout_prob =
    attention_probs_dropout_prob = 0.1), which the reference's from_pretrained models train
    with; the same keys in the YAML override them (0 = off), ``dropout_seed`` (default ``seed``)
    keys the counter-based masks."""
    return {"hidden_dropout": float(get(cfg, "hidden_dropout_prob", 0.1)),
            "attn_dropout": float(get(cfg, "attention_probs_dropout_prob", 0.1)),
            "dropout_seed": int(get(cfg, "dropout_seed", get(cfg, "seed", 0)))}


def mlm_finetune(cfg) -> Dict[str, object]:
    """MLM_PLL/main.py:117-161 (mlm_finetune_bert) on the native trainer (``train.MLMTrainer``).

    Reference keys (MLM_PLL/config/train.yaml): ``train_data_path`` / ``dev_data_path``
    (preprocessed do_job rows), ``num_of_data``, ``epoch``, ``lr``, ``dataloader.batch_size``
    (rows, 32), ``dataloader.shuffle`` (False), ``output_path``.  Batches are the reference's
    padded batches (``train.pad_rows``; CE over every position, [PAD] labels included); AdamW
    is re-created every epoch (``:76``); per epoch the dev loss (no update), then
    ``checkpoint_{epoch}.pth`` and ``loss.json`` (``{"train": [...], "dev": [...]}``, zeros for
    epochs not run yet, as ``:131-161`` writes it).  Extra: ``checkpoint_path`` /
    ``random_init_seed`` (initial weights: bert-base-chinese cannot be fetched offline),
    ``train_ref_text_path`` ({utt: text}, expanded by ``do_job_rows``), ``weight_decay``,
    dropout keys (``_dropout_args``).  ``dataloader.shuffle: True`` draws the order from torch.randperm seeded by ``seed`` (not the
    reference's sampler stream)."""
    import torch
    from .train import MLMTrainer, do_job_rows, mlm_epoch
    os.makedirs(cfg.output_path, exist_ok=True)
    n_data = int(get(cfg, "num_of_data", 1 << 62))

    def rows_of(split):
        rows_path, ref_path = get(cfg, f"{split}_data_path"), get(cfg, f"{split}_ref_text_path")
        if rows_path and os.path.exists(rows_path):
            rows = _load(rows_path)[:n_data]
            return [r["input_ids"] for r in rows], [r["labels"] for r in rows]
        if ref_path and os.path.exists(ref_path):
            refs = _load(ref_path)
            tok = _tokenizer(cfg, list(refs.values()))
            ids, off, lab = do_job_rows([[D.CLS_ID] + list(tok.encode_words(t)) + [D.SEP_ID] for t in refs.values()])
            n = min(len(off) - 1, n_data)
            return ([ids[off[i]:off[i + 1]].tolist() for i in range(n)],
                    [lab[off[i]:off[i + 1]].tolist() for i in range(n)])
        return None
    train_d, dev_d = rows_of("train"), rows_of("dev")
    if train_d is None:
        raise FileNotFoundError("train_data_path (do_job rows) or train_ref_text_path is required")
    tr = MLMTrainer(_weights(cfg, "mlm"), BERT_BASE, device=_dev(cfg), lr=float(get(cfg, "lr", 1e-5)),
                    weight_decay=float(get(cfg, "weight_decay", 0.01)), **_dropout_args(cfg))
    bs = int(get(cfg, "dataloader.batch_size", get(cfg, "batch_size", 32)))
    shuffle = bool(get(cfg, "dataloader.shuffle", False))
    gen = torch.Generator().manual_seed(int(get(cfg, "seed", 0)))
    epochs = int(get(cfg, "epoch", 1))
    train_rec, dev_rec, ckpts = [0] * epochs, [0] * epochs, []
    try:
        for ep in range(1, epochs + 1):
            tr.reset_optimizer()
            tr.set_dropout_step(ep << 32)            # epoch-keyed masks: a resumed run draws the same
            order = torch.randperm(len(train_d[0]), generator=gen).numpy() if shuffle else None
            train_rec[ep - 1] = mlm_epoch(tr, *train_d, bs, update=True, order=order)
            print("epoch ", ep, " train loss: ", train_rec[ep - 1])
            if dev_d is not None:
                dev_rec[ep - 1] = mlm_epoch(tr, *dev_d, bs, update="loss")
                print("epoch ", ep, " dev loss: ", dev_rec[ep - 1], "\n")
            ckpts.append(_save_checkpoint(cfg.output_path, tr.state_dict(), ep))
            D.json_saving(os.path.join(cfg.output_path, "loss.json"), {"train": train_rec, "dev": dev_rec})
    finally:
        tr.close()
    return {"train_loss": train_rec, "dev_loss": dev_rec, "checkpoints": ckpts}


def rescorebert(cfg) -> Dict[str, str]:
    """RescoreBert/main.py:232-285 (score): dev/test hyps -> CLS scores -> dev_lm/test_lm.json."""
    from .scorer import RescoreBertScorer
    sc = RescoreBertScorer(_weights(cfg, "cls"), BERT_BASE, device=_dev(cfg), max_rows=get(cfg, "max_rows", 65536),
                           precision=get(cfg, "precision", "fp16x3"))
    out_files = {}
    for split in ("dev", "test"):
        feats = get(cfg, f"{split}_feature", [])
        paths = get(cfg, f"{split}_feature_path", [])
        fmt = get(cfg, f"{split}_output_format")
        if "hyps_token_ids" not in feats or not fmt or not os.path.exists(fmt):
            continue
        hyps = _load(paths[feats.index("hyps_token_ids")])
        tok = _tokenizer(cfg, [t for h in hyps.values() for t in h.values()])
        max_utt, n_best = get(cfg, "max_utt", 1 << 30), get(cfg, "n_best", 1 << 30)
        nb, keys = _nbest_tokens(hyps, tok, max_utt, n_best)
        scores = sc.score(nb)
        out = D.get_output_format(fmt, max_utt, n_best)      # util/get_output_format.py:4-16
        for (u, h), s in zip(keys, scores):
            out[u][h] = float(s)
        path = os.path.join(cfg.output_path, f"{split}_lm.json")
        json_saving(path, out)
        out_files[split] = path
    sc.close()
    return out_files


def _rb_features(cfg, split: str):
    """RescoreBert/preprocess.py:8-55 get_feature: rows (utt, hyp) from the FIRST feature's
    JSON in key order (``max_utt`` utterances, ``n_best`` hypotheses each), then every named
    feature looked up per row: ``hyps_token_ids`` ([CLS] tokens [SEP] of the hypothesis text),
    ``mlm_pll_score``, ``hyps_am_score``, ``hyps_cer``.  Returns None without the split."""
    feats, paths = get(cfg, f"{split}_feature"), get(cfg, f"{split}_feature_path")
    if not feats or not paths:
        return None
    src = {f: _load(p) for f, p in zip(feats, paths)}
    max_utt, n_best = int(get(cfg, "max_utt", 1 << 30)), int(get(cfg, "n_best", 1 << 30))
    keys = []
    for u, (uid, hyps) in enumerate(src[feats[0]].items()):
        if u == max_utt:
            break
        for k, hid in enumerate(hyps):
            if k == n_best:
                break
            keys.append((uid, hid))
    out = {"keys": keys, "features": list(feats)}
    if "hyps_token_ids" in src:
        texts = src["hyps_token_ids"]
        tok = _tokenizer(cfg, [t for h in texts.values() for t in h.values()])
        seqs = [[D.CLS_ID] + list(tok.encode_words(texts[u][h])) + [D.SEP_ID] for u, h in keys]
        out["tokens"] = np.asarray([x for sq in seqs for x in sq], np.int32)
        out["hyp_off"] = np.concatenate([[0], np.cumsum([len(sq) for sq in seqs])]).astype(np.int32)
    for f in ("mlm_pll_score", "hyps_am_score", "hyps_cer"):
        if f in src:
            out[f] = np.asarray([src[f][u][h] for u, h in keys], np.float32)
    return out


def rescorebert_train(cfg) -> Dict[str, object]:
    """RescoreBert/main.py:166-229 (train) on the native trainer (``train.RescoreBertTrainer``).

    Reference keys (RescoreBert/config/MD*_train.yaml): ``method`` (MD / MD_MWER / MD_MWED),
    ``md_loss_weight``, ``lr``, ``epoch``, ``batch_size`` (utterances: batch_size * n_best
    rows), ``n_best``, ``max_utt``, ``train_feature`` / ``train_feature_path`` and ``dev_*``
    (hyps_token_ids = the hypothesis text JSON, mlm_pll_score, hyps_am_score, hyps_cer),
    ``output_path``, ``resume.start_from`` / ``resume.checkpoint_path``.  Per epoch: a fresh
    AdamW (``:83-86``), the train pass, the dev loss (no update), ``checkpoint_{epoch}.pth``
    and ``loss.json``.  Extra: ``checkpoint_path`` / ``random_init_seed`` (initial weights:
    bert-base-chinese cannot be fetched offline), ``weight_decay``, dropout keys (``_dropout_args``)."""
    from .train import RescoreBertTrainer, rescorebert_epoch
    os.makedirs(cfg.output_path, exist_ok=True)
    method = str(get(cfg, "method", "MD"))
    need = ["hyps_token_ids", "mlm_pll_score"] + (["hyps_am_score", "hyps_cer"] if method != "MD" else [])
    train_f, dev_f = _rb_features(cfg, "train"), _rb_features(cfg, "dev")
    for f in need:
        if train_f is None or f not in train_f["features"]:
            raise KeyError(f"train_feature must name {f} for method {method}")
    start = get(cfg, "resume.start_from")
    ck_resume = get(cfg, "resume.checkpoint_path")
    resume = start is not None and ck_resume is not None
    weights = load_state_dict_file(ck_resume) if resume else _weights(cfg, "cls")
    if resume:
        rec = _load(os.path.join(cfg.output_path, "loss.json"))
        train_rec, dev_rec = list(rec["train"]), list(rec["dev"])
    else:
        train_rec, dev_rec = [], []
    tr = RescoreBertTrainer(weights, BERT_BASE, device=_dev(cfg), method=method,
                            md_loss_weight=float(get(cfg, "md_loss_weight", 1.0)), lr=float(get(cfg, "lr", 1e-5)),
                            weight_decay=float(get(cfg, "weight_decay", 0.01)), **_dropout_args(cfg))
    bs, n_best = int(get(cfg, "batch_size", 1)), int(get(cfg, "n_best", 1))

    def epoch_pass(f, update):
        z = np.zeros(len(f["hyp_off"]) - 1, np.float32)
        return rescorebert_epoch(tr, f["tokens"], f["hyp_off"], f["mlm_pll_score"], f.get("hyps_am_score", z),
                                 f.get("hyps_cer", z), bs, n_best, update=update)
    ckpts = []
    try:
        for ep in range(int(start) if resume else 1, int(get(cfg, "epoch", 1)) + 1):
            print("Epoch {}/{}".format(ep, get(cfg, "epoch", 1)))
            tr.reset_optimizer()
            tr.set_dropout_step(ep << 32)            # epoch-keyed masks: a resumed run draws the same
            train_rec.append(epoch_pass(train_f, True))
            print("epoch ", ep, " train loss: ", train_rec[-1], "\n")
            if dev_f is not None and all(f in dev_f["features"] for f in need):
                dev_rec.append(epoch_pass(dev_f, "loss"))
                print("epoch ", ep, " dev loss: ", dev_rec[-1], "\n")
            ckpts.append(_save_checkpoint(cfg.output_path, tr.state_dict(), ep))
            D.json_saving(os.path.join(cfg.output_path, "loss.json"), {"train": train_rec, "dev": dev_rec})
    finally:
        tr.close()
    return {"train_loss": train_rec, "dev_loss": dev_rec, "checkpoints": ckpts}


def rescore(cfg) -> Dict[str, float]:
    """rescore.py:61-120: best weight on dev, CER on test, logged to output_path/rescore.log."""
    from . import rerank
    os.makedirs(cfg.output_path, exist_ok=True)
    log = _logger(os.path.join(cfg.output_path, "rescore.log"))
    log.info(str(cfg))
    mode = get(cfg, "mode", "norm")
    n_best = cfg.n_best

    def split_nb(prefix):
        hyps = _load(getattr(cfg, f"{prefix}_hyps_text_path"))
        refs = _load(getattr(cfg, f"{prefix}_ref_text_path"))
        am = _load(getattr(cfg, f"{prefix}_am_path"))
        lm_j = _load(getattr(cfg, f"{prefix}_lm_path"))
        nb = D.from_texts(hyps, refs, am, n_best=n_best)
        lm = np.asarray([lm_j[u][h] for u in nb.utt_ids for h in list(lm_j[u])[:n_best]], np.float64)
        return nb, lm

    dev_nb, dev_lm = split_nb("dev")
    best_w, best_cer, _, _ = rerank.find_best_weight(dev_nb, dev_lm, n_best=n_best, mode=mode, device=_dev(cfg))
    log.info("best_weight: " + str(best_w))
    log.info("dev cer: " + str(best_cer))
    print("best_weight: ", best_w)
    print("dev cer: ", best_cer)
    test_nb, test_lm = split_nb("test")
    arg = rerank.fuse_rerank(test_nb.am, test_lm, test_nb.hyp_len(), test_nb.utt_off, [best_w], mode, n_best,
                             device=_dev(cfg))
    ed = rerank.ref_edits(test_nb, device=_dev(cfg))
    edits = rerank.corpus_edits(ed, test_nb.utt_off, arg).cpu().numpy()[0]
    test_cer = float(edits) / sum(len(r) for r in test_nb.refs)
    log.info("test cer: " + str(test_cer))
    print("test cer: ", test_cer)
    return {"best_weight": best_w, "dev_cer": best_cer, "test_cer": test_cer}


def rmbr(cfg) -> Dict[str, float]:
    """RMBR/main.py:38-108; utility_function: cer (RMBR/utility_functions.py:28-33) or
    bertscore (:9-22, bert_score restated on the HIP path: ``bertscore.BertScorer``, weights
    from checkpoint_path / random_init_seed, ``bertscore_layers`` (8), ``bertscore_component``
    (P / R / F, default R))."""
    from . import rerank
    util = str(get(cfg, "utility_function", "cer")).lower().replace("_", "")
    if util not in ("cer", "bertscore"):
        raise ValueError(f"unknown utility_function {util!r} (cer, bertscore)")
    os.makedirs(cfg.output_path, exist_ok=True)
    log = _logger(os.path.join(cfg.output_path, "mbr.log"))
    n_best, max_utt = cfg.n_best, get(cfg, "max_utt", 1 << 30)
    scorer = tok = None
    if util == "bertscore":
        from . import bertscore as BS
        scorer = BS.BertScorer(_weights(cfg, "mlm"), BERT_BASE, num_layers=get(cfg, "bertscore_layers", 8),
                               device=_dev(cfg), max_rows=get(cfg, "max_rows", 65536),
                               precision=get(cfg, "precision", "fp16x3"))
        which = str(get(cfg, "bertscore_component", "R")).upper()
        bs_batch = int(get(cfg, "batch_size", 128))     # RMBR/config/RMBR.yaml: bert_score batch_size

    def split_nb(prefix):
        nonlocal tok
        feats, paths = getattr(cfg, f"{prefix}_feature"), getattr(cfg, f"{prefix}_feature_path")
        refs = _load(paths[feats.index("ref_text")])
        hyps = _load(paths[feats.index("hyps_text")])
        nb = D.from_texts(hyps, refs, None, n_best=n_best, max_utt=max_utt)
        if scorer is None:
            return nb, None
        if tok is None:
            tok = _tokenizer(cfg, [t for h in hyps.values() for t in h.values()])
        return nb, _nbest_tokens(hyps, tok, max_utt, n_best)[0]

    def decode(nb, nb_tok, k):
        if scorer is None:
            return rerank.mbr_decode(nb, k, device=_dev(cfg))
        return BS.mbr_decode(scorer, nb_tok, k, which, batch_size=bs_batch)

    dev, dev_tok = split_nb("dev")
    log.info("Running MBR on dev set to find best length ...")
    if scorer is None:
        best_cer, best_len, best_sc = rerank.find_best_length(dev, n_best, device=_dev(cfg))
    else:
        best_cer, best_len, best_sc = BS.find_best_length(scorer, dev_tok, n_best, which, nb_chars=dev,
                                                          batch_size=bs_batch)
    log.info(f"best_cer: {best_cer}")
    log.info(f"best_length: {best_len}")
    print("best_cer: ", best_cer)
    print("best_length: ", best_len)
    res = {"best_cer": best_cer, "best_length": best_len}
    for split, nb, sc in (("dev", dev, best_sc), ("test", None, None)):
        if split == "test":
            nb, nb_tok = split_nb("test")
            log.info("Running MBR on test set ...")
            idx, sc = decode(nb, nb_tok, best_len)
            import torch
            ed = rerank.ref_edits(nb, device=_dev(cfg))
            arg = torch.from_numpy(idx.astype(np.int32)).to(ed.device)[None, :]
            test_cer = float(rerank.corpus_edits(ed, nb.utt_off, arg).cpu()[0]) / sum(len(r) for r in nb.refs)
            log.info(f"test cer: {test_cer}")
            print("test cer: ", test_cer)
            res["test_cer"] = test_cer
        fmt = getattr(cfg, f"{split}_output_format")
        out = D.get_output_format(fmt, max_utt, n_best)
        for (uid, hyps), row in zip(out.items(), sc.tolist()):   # RMBR/main.py:80-89
            for (hid, _), v in zip(hyps.items(), row):
                out[uid][hid] = v
        D.json_saving(os.path.join(cfg.output_path, f"{split}_MBR.json"), out)
    if scorer is not None:
        scorer.close()
    return res


def _dev(cfg) -> int:
    d = str(get(cfg, "device", "cuda:0"))
    return int(d.split(":")[1]) if ":" in d else 0


def _logger(path):
    log = logging.getLogger("asr_rescoring_amd." + os.path.basename(path))
    log.setLevel(logging.INFO)
    h = logging.FileHandler(path, mode="w")
    h.setFormatter(logging.Formatter("%(asctime)s,%(msecs)d %(name)s %(levelname)s %(message)s", "%H:%M:%S"))
    log.handlers = [h]
    return log


COMMANDS = {"mlm_pll": mlm_pll, "mlm_finetune": mlm_finetune, "rescorebert": rescorebert,
            "rescorebert_train": rescorebert_train,
            "rescore": rescore, "rmbr": rmbr}


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] not in COMMANDS:
        print("usage: python -m asr_rescoring_amd.cli {" + ",".join(COMMANDS) + "} --config <yaml>")
        return 2
    cfg = ArgParser().parse(argv[1:])
    COMMANDS[argv[0]](cfg)
    return 0


if __name__ == "__main__":
    sys.exit(main())

