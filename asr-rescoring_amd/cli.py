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
    if world == 1:
        allv = scorer.row_logprobs(rows).cpu().tolist() if rows else []
        for r, s in zip(rows, allv):
            output_score[r["utt_id"]][r["hyp_id"]] += s
        return output_score
    import torch.distributed as dist
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


def mlm_finetune(cfg) -> Dict[str, object]:
    """MLM_PLL/main.py:117-161 (mlm_finetune_bert) on the native trainer (``train.MLMTrainer``).

    Data: ``train_data_path`` (preprocessed ``do_job`` rows: input_ids / labels) or
    ``train_ref_text_path`` ({utt: text}; tokenised and expanded by ``do_job_rows``).  Keys:
    ``epochs``, ``batch_size`` (rows per step, 32), ``lr``, ``weight_decay``, ``shuffle`` +
    ``seed``; AdamW is re-created every epoch as the reference does (``:76``,
    ``reset_optimizer`` false keeps it).  Writes ``checkpoint_{epoch}.pt`` per epoch (``:157``)."""
    import torch
    from .train import MLMTrainer, do_job_rows
    os.makedirs(cfg.output_path, exist_ok=True)
    log = _logger(os.path.join(cfg.output_path, "train.log"))
    rows_path, ref_path = get(cfg, "train_data_path"), get(cfg, "train_ref_text_path")
    if rows_path and os.path.exists(rows_path):
        rows = _load(rows_path)
        seqs = [r["input_ids"] for r in rows]
        labs = [r["labels"] for r in rows]
    else:
        refs = _load(ref_path)
        tok = _tokenizer(cfg, list(refs.values()))
        hyps = [[101] + list(tok.encode_words(t)) + [102] for t in refs.values()]
        ids, off, lab = do_job_rows(hyps)
        seqs = [ids[off[i]:off[i + 1]].tolist() for i in range(len(off) - 1)]
        labs = [lab[off[i]:off[i + 1]].tolist() for i in range(len(off) - 1)]
    tr = MLMTrainer(_weights(cfg, "mlm"), BERT_BASE, device=_dev(cfg), lr=float(get(cfg, "lr", 1e-5)),
                    weight_decay=float(get(cfg, "weight_decay", 0.01)))
    bs = int(get(cfg, "batch_size", 32))
    rng = np.random.default_rng(int(get(cfg, "seed", 0)))
    losses, ckpts = [], []
    for ep in range(int(get(cfg, "epochs", 1))):
        if ep and get(cfg, "reset_optimizer", True):
            tr.reset_optimizer()
        order = rng.permutation(len(seqs)) if get(cfg, "shuffle", True) else np.arange(len(seqs))
        tot, nb_ = 0.0, 0
        for b0 in range(0, len(order), bs):
            idx = order[b0:b0 + bs]
            off = np.zeros(len(idx) + 1, np.int32)
            off[1:] = np.cumsum([len(seqs[i]) for i in idx])
            ids = np.concatenate([np.asarray(seqs[i], np.int32) for i in idx])
            lab = np.concatenate([np.asarray(labs[i], np.int32) for i in idx])
            tot += tr.step(ids, off, lab)
            nb_ += 1
        losses.append(tot / max(nb_, 1))
        log.info(f"epoch {ep + 1} loss {losses[-1]}")
        path = os.path.join(cfg.output_path, f"checkpoint_{ep + 1}.pt")
        torch.save({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in tr.state_dict().items()}, path)
        ckpts.append(path)
    tr.close()
    return {"losses": losses, "checkpoints": ckpts}


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


def rescorebert_train(cfg) -> Dict[str, object]:
    """RescoreBert/main.py:166-229 (train) on the native trainer (``train.RescoreBertTrainer``).

    ``train_feature`` / ``train_feature_path`` name ``hyps_text``, ``ref_text``, ``hyps_score``
    (AM) and ``mlm_score`` (the MLM_PLL teacher JSON written by ``mlm_pll``).  Keys:
    ``loss_type`` (MD / MD_MWER / MD_MWED), ``lambda``, ``epochs``, ``batch_size``
    (utterances per step), ``lr``, ``weight_decay``, ``n_best``, ``reset_optimizer`` (a fresh
    AdamW each epoch).  Writes ``checkpoint_{epoch}.pt`` (HF keys, torch.save of tensors:
    loadable with ``torch.load(weights_only=True)`` as ``checkpoint_path``) and ``train.log``."""
    import torch
    from . import rerank
    from .train import RescoreBertTrainer
    os.makedirs(cfg.output_path, exist_ok=True)
    log = _logger(os.path.join(cfg.output_path, "train.log"))
    feats, paths = cfg.train_feature, cfg.train_feature_path
    src = {f: _load(p) for f, p in zip(feats, paths)}
    n_best, max_utt = get(cfg, "n_best", 1 << 30), get(cfg, "max_utt", 1 << 30)
    hyps = src["hyps_text"]
    nb_c = D.from_texts(hyps, src["ref_text"], src["hyps_score"], n_best=n_best, max_utt=max_utt)
    tok = _tokenizer(cfg, [t for h in hyps.values() for t in h.values()])
    nb, keys = _nbest_tokens(hyps, tok, max_utt, n_best)
    target = np.asarray([src["mlm_score"][u][h] for u, h in keys], np.float32)
    err = rerank.ref_edits(nb_c, device=_dev(cfg)).cpu().numpy().astype(np.float32)
    am = nb_c.am.astype(np.float32)
    tr = RescoreBertTrainer(_weights(cfg, "cls"), BERT_BASE, device=_dev(cfg), loss=get(cfg, "loss_type", "MD"),
                            lam=float(get(cfg, "lambda", 1.0)), lr=float(get(cfg, "lr", 1e-5)),
                            weight_decay=float(get(cfg, "weight_decay", 0.01)))
    bs = int(get(cfg, "batch_size", 3))
    losses, ckpts = [], []
    for ep in range(int(get(cfg, "epochs", 1))):
        if ep and get(cfg, "reset_optimizer", False):
            tr.reset_optimizer()
        tot = 0.0
        for b0 in range(0, nb.n_utt, bs):
            utts = list(range(b0, min(nb.n_utt, b0 + bs)))
            sub = nb.subset(utts)
            h0, h1 = nb.utt_off[utts[0]], nb.utt_off[utts[-1] + 1]
            loss, _ = tr.step(sub.tokens, sub.hyp_off, sub.utt_off, target[h0:h1], am[h0:h1], err[h0:h1])
            tot += loss
        losses.append(tot / max(1, -(-nb.n_utt // bs)))
        log.info(f"epoch {ep + 1} loss {losses[-1]}")
        path = os.path.join(cfg.output_path, f"checkpoint_{ep + 1}.pt")
        torch.save({k: torch.from_numpy(v) for k, v in tr.state_dict().items()}, path)
        ckpts.append(path)
    tr.close()
    return {"losses": losses, "checkpoints": ckpts}


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
        return BS.mbr_decode(scorer, nb_tok, k, which)

    dev, dev_tok = split_nb("dev")
    log.info("Running MBR on dev set to find best length ...")
    if scorer is None:
        best_cer, best_len, best_sc = rerank.find_best_length(dev, n_best, device=_dev(cfg))
    else:
        best_cer, best_len, best_sc = BS.find_best_length(scorer, dev_tok, n_best, which, nb_chars=dev)
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

