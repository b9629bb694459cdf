"""GPU parity at the shapes of BASELINE.json's configs (C2, C3, C5), and the reference's
own drop-in entry points on the reference's own input formats.

* C3 (MLM_PLL full PLL, bert-base, N=50, L ~ U{24..40}): 6 utterances x 50 hypotheses,
  HIP vs the oracle's fp32 restatement of run_one_epoch (MLM_PLL/main.py:73-114): every
  masked row and every PLL within 1e-3 relative; then the 101-weight fusion sweep of
  rescore.py:25-58 fed the ORACLE's lm and fed the HIP lm gives the same argmax for every
  weight, the same best weight and the same CER (the north-star rerank-index check).  The
  "hard" synthetic variant (reference hypothesis not first, AM unsorted) makes the argmax
  move with the weight.
* C4 (MLM_PLL, N=100, real alfred lengths): 2 utterances x 100 plus a T > 64 utterance in one
  launch chunk (mixed attention kernels), rows / PLL / rerank argmax vs the oracle, and
  ``cli mlm_pll`` as 1 rank vs 2 ranks bitwise.
* C2 (RescoreBert, N=50): 10 utterances x 50 hypotheses vs the oracle's RescoreBert batches.
* C5 (RMBR CER utility + fusion, N=100, real lengths): 3 utterances x 100 hypotheses, the
  pairwise edit matrices, MBR scores for several k (float32, bit-exact) and the fusion argmax
  for all 101 weights vs the oracle.
* PLLScorer.run_one_epoch and ``cli mlm_pll`` with ``train_data_path`` on do_job rows
  (MLM_PLL/preprocess.py:9-30 format), and ``cli rescorebert`` on a hyps JSON, against the
  reference-run F1 / F2 fixtures.
"""
import json
import os

import numpy as np
import pytest
import yaml

from asr_rescoring_amd import data as D
from asr_rescoring_amd.weights import BERT_BASE, make_weights

pytestmark = pytest.mark.gpu

REL = 1e-3


def rel_err(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.abs(a - b) / np.maximum(np.abs(b), 1e-30)


@pytest.fixture(scope="module")
def w_base():
    return make_weights(BERT_BASE, seed=1234, with_cls_linear=True, with_pooler=True)


@pytest.fixture(scope="module")
def oracle_model(w_base):
    from oracle.bert_ref import TorchBert, set_cpu_threads
    set_cpu_threads()
    return TorchBert(w_base, BERT_BASE)


def _lengths(golden_dir):
    lc = json.load(open(os.path.join(golden_dir, "alfred_test_lengths.json")))["length_counts"]
    return np.repeat(np.arange(len(lc)), lc).astype(np.int64)


def _oracle_hyps(nb):
    U = nb.n_utt
    N = int(np.diff(nb.utt_off)[0])
    return [[nb.hyp_words(nb.utt_off[u] + i) for i in range(N)] for u in range(U)], N


def test_c3_shape_pll_rows_and_rerank(w_base, oracle_model):
    from asr_rescoring_amd.scorer import PLLScorer
    from asr_rescoring_amd import rerank
    from oracle import rescore_ref as RR
    from oracle.bert_ref import pll_reference_pattern
    nb = D.synthetic_nbest(6, 50, seed=31, hard=True)
    s = PLLScorer(w_base, BERT_BASE, device=0, max_rows=65536)
    try:
        pll, rows = s.score_nbest(nb.tokens, nb.hyp_off, return_rows=True)
        pll, rows = pll.cpu().numpy(), rows.cpu().numpy()
    finally:
        s.close()
    ref_rows, ref_pll = pll_reference_pattern(oracle_model, nb.tokens, nb.hyp_off, batch_size=64,
                                              full_head=False)
    assert len(rows) == len(ref_rows) == nb.n_forwards()
    er = rel_err(rows, ref_rows)
    assert er.max() < REL, er.max()
    assert rel_err(pll, ref_pll).max() < REL
    # fusion sweep: oracle fed its own lm vs fed the HIP lm (rescore.py:25-58)
    hyps, N = _oracle_hyps(nb)
    am = nb.am.reshape(nb.n_utt, N)
    bw_o, cer_o, arg_o = RR.find_best_weight(am, ref_pll.reshape(nb.n_utt, N), hyps, nb.refs, n_best=N)
    bw_h, cer_h, arg_h = RR.find_best_weight(am, pll.reshape(nb.n_utt, N), hyps, nb.refs, n_best=N)
    assert np.array_equal(arg_o, arg_h) and bw_o == bw_h and cer_o == cer_h
    assert len({tuple(a) for a in arg_o}) > 1, "the argmax never moved: the check would be vacuous"
    # and the HIP fusion + CER kernels on the HIP lm equal the oracle on the same lm
    bw_g, cer_g, arg_g, _ = rerank.find_best_weight(nb, pll, n_best=N)
    assert np.array_equal(arg_g, arg_h) and bw_g == bw_h and cer_g == cer_h


def test_c3_finetuned_lm_moves_the_pick(w_base):
    """The reference's pipeline on the C3 shape: MLM fine-tuning on in-domain text
    (MLM_PLL/main.py:117-161; here the utterances' reference sentences, the native trainer, 300
    deterministic steps) -> scoring with that checkpoint (:184-186) -> fusion (rescore.py:25-58).
    With this LM the best weight is > 0 and the reranked CER is below the AM-only CER, so the
    101-weight argmax equality between the oracle's lm and the HIP lm is checked where the LM
    actually moves the pick."""
    from asr_rescoring_amd.scorer import PLLScorer
    from asr_rescoring_amd import rerank
    from asr_rescoring_amd.train import finetune_mlm_on_texts
    from oracle import rescore_ref as RR
    from oracle.bert_ref import TorchBert, pll_reference_pattern
    nb = D.synthetic_nbest(6, 50, seed=31, hard=True)
    w_ft, losses = finetune_mlm_on_texts(w_base, nb.refs, BERT_BASE, steps=300, lr=1e-4, seed=0, device=0)
    assert np.isfinite(losses).all()
    s = PLLScorer(w_ft, BERT_BASE, device=0, max_rows=65536)
    try:
        pll = s.score_nbest(nb.tokens, nb.hyp_off).cpu().numpy()
    finally:
        s.close()
    _, ref_pll = pll_reference_pattern(TorchBert(w_ft, BERT_BASE), nb.tokens, nb.hyp_off, batch_size=64,
                                       full_head=False)
    assert rel_err(pll, ref_pll).max() < REL
    hyps, N = _oracle_hyps(nb)
    am = nb.am.reshape(nb.n_utt, N)
    bw_o, cer_o, arg_o = RR.find_best_weight(am, ref_pll.reshape(nb.n_utt, N), hyps, nb.refs, n_best=N)
    bw_h, cer_h, arg_h = RR.find_best_weight(am, pll.reshape(nb.n_utt, N), hyps, nb.refs, n_best=N)
    assert np.array_equal(arg_o, arg_h) and bw_o == bw_h and cer_o == cer_h
    bw_g, cer_g, arg_g, cers = rerank.find_best_weight(nb, pll, n_best=N)
    assert np.array_equal(arg_g, arg_h) and bw_g == bw_h and cer_g == cer_h
    assert bw_h > 0 and cer_h < cers[0], (bw_h, cer_h, cers[0])


def test_c3_50_utterances_finetuned_vs_torch_fp32_on_gpu(w_base):
    """Wider scoring parity at the C3 shape: 50 utterances x N=50 (about 80k masked forwards) with
    a fine-tuned LM (the reference's fine-tune -> score -> fuse pipeline, MLM_PLL/main.py:117-161,
    :184-186, rescore.py:25-45), against the same restatement run as a plain torch fp32 reference on
    the GPU (the CPU oracle would take an hour at this size): PLL within 1e-3 (fp32-class: ~1e-6),
    the 101-weight argmax and corpus CER equal for every utterance, and the LM moves the pick."""
    import torch
    from asr_rescoring_amd.scorer import PLLScorer
    from asr_rescoring_amd.train import finetune_mlm_on_texts
    from oracle import rescore_ref as RR
    from oracle.bert_ref import TorchBert, pll_reference_pattern
    nb = D.synthetic_nbest(50, 50, seed=7, hard=True)
    w_ft, _ = finetune_mlm_on_texts(w_base, nb.refs, BERT_BASE, steps=300, lr=1e-4, seed=0, device=0)
    s = PLLScorer(w_ft, BERT_BASE, device=0, max_rows=262144)
    try:
        pll = s.score_nbest(nb.tokens, nb.hyp_off).cpu().numpy()
    finally:
        s.close()
    prev = torch.backends.cuda.matmul.allow_tf32
    torch.backends.cuda.matmul.allow_tf32 = False
    try:
        _, ref_pll = pll_reference_pattern(TorchBert(w_ft, BERT_BASE, device="cuda"), nb.tokens, nb.hyp_off,
                                           batch_size=512, full_head=False)
    finally:
        torch.backends.cuda.matmul.allow_tf32 = prev
    assert rel_err(pll, ref_pll).max() < REL
    hyps, N = _oracle_hyps(nb)
    am = nb.am.reshape(nb.n_utt, N)
    bw_o, cer_o, arg_o = RR.find_best_weight(am, ref_pll.reshape(nb.n_utt, N), hyps, nb.refs, n_best=N)
    bw_h, cer_h, arg_h = RR.find_best_weight(am, pll.reshape(nb.n_utt, N), hyps, nb.refs, n_best=N)
    assert np.array_equal(arg_o, arg_h) and bw_o == bw_h and cer_o == cer_h
    am_only = RR.corpus_cer(nb.refs, [utt[i] for utt, i in zip(hyps, arg_h[0])])      # weight 0
    assert bw_h > 0 and cer_h < am_only, (bw_h, cer_h, am_only)


def test_c2_shape_cls(w_base, oracle_model):
    import torch
    from asr_rescoring_amd.scorer import RescoreBertHIP
    from oracle.bert_ref import cls_reference_pattern
    nb = D.synthetic_nbest(10, 50, seed=32)
    ref = cls_reference_pattern(oracle_model, nb.tokens, nb.hyp_off, batch_rows=150, with_pooler=True)
    m = RescoreBertHIP(w_base, BERT_BASE, device=0, max_rows=65536)
    try:
        got = m.engine.score_nbest(nb.tokens, nb.hyp_off).cpu().numpy()
        # the nn.Module drop-in on one reference batch (batch_size 3 x n_best 50 rows, padded)
        seqs = [torch.tensor(nb.tokens[nb.hyp_off[h]:nb.hyp_off[h + 1]], dtype=torch.long) for h in range(150)]
        ids = torch.nn.utils.rnn.pad_sequence(seqs, batch_first=True)
        msk = torch.nn.utils.rnn.pad_sequence([torch.ones_like(x) for x in seqs], batch_first=True)
        mod = m(ids.cuda(), msk.cuda()).cpu().numpy()
    finally:
        m.engine.close()
    err = np.abs(got - ref)
    assert (err <= np.maximum(REL * np.abs(ref), 1e-4)).all(), err.max()
    assert np.array_equal(mod, got[:150])


def test_c5_shape_rmbr_and_fusion(golden_dir):
    import torch
    from asr_rescoring_amd import rerank
    from oracle import rescore_ref as RR
    nb = D.synthetic_nbest(3, 100, seed=33, lengths=_lengths(golden_dir), hard=True)
    hyps, N = _oracle_hyps(nb)
    ed, moff = rerank.pairwise_edit(nb)
    ed = ed.cpu().numpy()
    for u in range(nb.n_utt):
        m = ed[moff[u]:moff[u + 1]].reshape(N, N)
        want = np.array([[RR.levenshtein(hyps[u][i], hyps[u][j]) for j in range(N)] for i in range(N)])
        assert np.array_equal(m, want)
    ed_d = torch.from_numpy(ed).cuda()
    for k in (2, 7, 50, 100):
        arg, sc = rerank.mbr_scores(nb, k, ed_d, moff)
        oarg, osc = RR.mbr_decode(k, hyps)
        assert np.array_equal(sc, osc) and np.array_equal(arg, oarg), k
    # LM-score fusion over the 101-weight grid at N=100 (rescore.py:47-58), fp64 bit-exact
    rng = np.random.default_rng(5)
    lm = -np.abs(rng.normal(60.0, 20.0, size=nb.n_hyp))
    for mode in ("norm", "legacy", "am_norm"):
        grid = rerank.weight_grid(mode)
        arg = rerank.fuse_rerank(nb.am, lm, nb.hyp_len(), nb.utt_off, grid, mode, N).cpu().numpy()
        lens = nb.hyp_len().reshape(nb.n_utt, N)
        want = np.stack([np.argmax(RR.fuse(w, lens, nb.am.reshape(nb.n_utt, N), lm.reshape(nb.n_utt, N), mode),
                                   axis=-1) for w in grid])
        assert np.array_equal(arg, want), mode


def _do_job_rows(g):
    """The reference's preprocessed rows (MLM_PLL/preprocess.py:9-30) for the F1 fixture."""
    rows = []
    for u in range(len(g["utt_off"]) - 1):
        for k, h in enumerate(range(g["utt_off"][u], g["utt_off"][u + 1])):
            seq = [int(x) for x in g["tokens"][g["hyp_off"][h]:g["hyp_off"][h + 1]]]
            for p in range(1, len(seq) - 1):
                ids = list(seq)
                ids[p] = 103
                rows.append({"utt_id": f"utt{u}", "hyp_id": f"hyp_{k + 1}", "input_ids": ids,
                             "attention_masks": [1] * len(seq), "mask_pos": p, "labels": seq})
    return rows


def _load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name), allow_pickle=False)


def test_run_one_epoch_do_job_rows(w_base, golden_dir):
    from asr_rescoring_amd.scorer import PLLScorer
    g = _load(golden_dir, "pll_base.npz")
    rows = _do_job_rows(g)
    out = {}
    for r in rows:                                  # MLM_PLL/main.py:189-193
        if r["hyp_id"] == "hyp_1":
            out[r["utt_id"]] = {}
        out[r["utt_id"]][r["hyp_id"]] = 0
    s = PLLScorer(w_base, BERT_BASE, device=0, max_rows=8192)
    try:
        out = s.run_one_epoch(rows, out)
    finally:
        s.close()
    got = np.array([v for u in out.values() for v in u.values()])
    assert rel_err(got, g["pll"]).max() < REL


def test_cli_mlm_pll_data_path(golden_dir, tmp_path):
    from asr_rescoring_amd import cli
    g = _load(golden_dir, "pll_base.npz")
    rows = _do_job_rows(g)
    json.dump(rows, open(tmp_path / "train_rows.json", "w"))
    cfg = tmp_path / "score.yaml"
    cfg.write_text(yaml.safe_dump({"task": "scoring", "device": "cuda:0", "random_init_seed": 1234,
                                   "train_data_path": str(tmp_path / "train_rows.json"),
                                   "output_path": str(tmp_path) + "/", "model": {"bert": "bert-base-chinese"}}))
    assert cli.main(["mlm_pll", "--config", str(cfg)]) == 0
    lm = json.load(open(tmp_path / "train_lm.json"))
    assert list(lm) == [f"utt{u}" for u in range(len(g["utt_off"]) - 1)]
    got = np.array([v for u in lm.values() for v in u.values()])
    assert rel_err(got, g["pll"]).max() < REL


def test_cli_rescorebert_vs_f2(golden_dir, tmp_path):
    """cli rescorebert (RescoreBert/main.py:232-285) on a hyps JSON whose characters map to
    the F2 token ids through a vocab.txt: dev_lm.json equals the reference-run F2 scores."""
    from asr_rescoring_amd import cli
    g = _load(golden_dir, "cls_base.npz")
    tok, off = g["tokens"], g["hyp_off"]
    used = sorted({int(t) for t in tok if t >= 106})
    ch = {t: chr(0x4E00 + i) for i, t in enumerate(used)}
    special = {0: "[PAD]", 100: "[UNK]", 101: "[CLS]", 102: "[SEP]", 103: "[MASK]"}
    vocab = [special.get(i, ch.get(i, f"[unused{i}]")) for i in range(BERT_BASE.vocab)]
    (tmp_path / "vocab.txt").write_text("\n".join(vocab) + "\n", encoding="utf-8")
    hyps, fmt = {}, {}
    n_hyp = len(off) - 1
    per_utt = 4
    for h in range(n_hyp):
        u, k = divmod(h, per_utt)
        text = "".join(ch[int(t)] for t in tok[off[h] + 1:off[h + 1] - 1])
        hyps.setdefault(f"utt{u}", {})[f"hyp_{k + 1}"] = text
        fmt.setdefault(f"utt{u}", {})[f"hyp_{k + 1}"] = 0.0
    json.dump(hyps, open(tmp_path / "hyps.json", "w", encoding="utf-8"), ensure_ascii=False)
    json.dump(fmt, open(tmp_path / "fmt.json", "w", encoding="utf-8"))
    cfg = tmp_path / "MD_score.yaml"
    cfg.write_text(yaml.safe_dump({
        "device": "cuda:0", "random_init_seed": 1234, "n_best": per_utt,
        "model": {"bert": "bert-base-chinese", "vocab": str(tmp_path / "vocab.txt")},
        "dev_feature": ["hyps_token_ids"], "dev_feature_path": [str(tmp_path / "hyps.json")],
        "dev_output_format": str(tmp_path / "fmt.json"), "output_path": str(tmp_path)}, allow_unicode=True))
    files = cli.rescorebert(cli.ArgParser().parse(["--config", str(cfg)]))
    lm = json.load(open(files["dev"], encoding="utf-8"))
    got = np.array([v for u in lm.values() for v in u.values()], np.float64)
    err = np.abs(got - g["cls"])
    assert (err <= np.maximum(REL * np.abs(g["cls"]), 1e-4)).all(), err.max()


def _concat(parts):
    """One NBest of several (utterances in order)."""
    toks, hoff, uoff, am, refs, uids, hids = [], [0], [0], [], [], [], []
    for nb in parts:
        toks.append(nb.tokens)
        hoff.extend((np.asarray(nb.hyp_off[1:], np.int64) + hoff[-1]).tolist())
        uoff.extend((np.asarray(nb.utt_off[1:], np.int64) + uoff[-1]).tolist())
        am.append(nb.am)
        refs += nb.refs
        hids += nb.hyp_ids
    uids = [f"utt_{u}" for u in range(len(uoff) - 1)]
    return D.NBest(np.concatenate(toks).astype(np.int32), np.asarray(hoff, np.int32), np.asarray(uoff, np.int32),
                   np.concatenate(am), refs, uids, hids)


def test_c4_shape_real_lengths_mixed_chunk_and_ranks(w_base, oracle_model, golden_dir, tmp_path):
    """C4 (MLM_PLL utterance-sharded, full dev set, N=100; MLM_PLL/main.py:164-203) at test
    scale: 2 utterances x N=100 with base lengths drawn from the alfred test histogram
    (mean T ~17; its longest reference has 37 characters, so every C4 sequence has T <= 64),
    plus one utterance of T ~ 68-72 hypotheses scored in the SAME launch chunk, so the chunk
    mixes T <= 64 sequences (16x16 attention) with T > 64 ones (online-softmax attention) and
    layer-0 dedup is off for it.  Every masked row and PLL within 1e-3 of the oracle; the
    101-weight fusion argmax from the oracle's lm equals the one from the HIP lm for the two
    N=100 utterances; ``cli mlm_pll`` on the same texts as 1 rank and as 2 ranks (gloo
    exchange, both on this GPU) writes bitwise-equal scores that match the scorer's."""
    import socket
    import subprocess
    import sys
    import yaml
    from conftest import REPO
    from asr_rescoring_amd.scorer import PLLScorer
    from oracle import rescore_ref as RR
    from oracle.bert_ref import pll_reference_pattern
    nb_a = D.synthetic_nbest(2, 100, seed=41, lengths=_lengths(golden_dir), hard=True)
    nb_b = D.synthetic_nbest(1, 10, seed=42, len_lo=66, len_hi=70, hard=True)
    nb = _concat([nb_a, nb_b])
    T = np.diff(nb.hyp_off)
    assert T[:200].max() <= 64 < T[200:].min()
    assert int(((T - 2) * T).sum()) <= 131072      # one launch chunk
    s = PLLScorer(w_base, BERT_BASE, device=0, max_rows=131072)
    try:
        pll, rows = s.score_nbest(nb.tokens, nb.hyp_off, return_rows=True)
        pll, rows = pll.cpu().numpy(), rows.cpu().numpy()
    finally:
        s.close()
    ref_rows, ref_pll = pll_reference_pattern(oracle_model, nb.tokens, nb.hyp_off, batch_size=64,
                                              full_head=False)
    assert rel_err(rows, ref_rows).max() < REL
    assert rel_err(pll, ref_pll).max() < REL
    hyps, N = _oracle_hyps(nb_a)
    am = nb_a.am.reshape(nb_a.n_utt, N)
    bw_o, cer_o, arg_o = RR.find_best_weight(am, ref_pll[:200].reshape(2, N), hyps, nb_a.refs, n_best=N)
    bw_h, cer_h, arg_h = RR.find_best_weight(am, pll[:200].reshape(2, N), hyps, nb_a.refs, n_best=N)
    assert np.array_equal(arg_o, arg_h) and bw_o == bw_h and cer_o == cer_h
    assert len({tuple(a) for a in arg_o}) > 1, "the argmax never moved: the check would be vacuous"

    # cli mlm_pll (text -> native BertTokenizer-compatible tokenizer -> sharded scoring)
    used = sorted({int(t) for t in nb.tokens if t >= D.FIRST_WORD_ID})
    ch = {t: chr(0x4E00 + t - D.FIRST_WORD_ID) for t in used}
    special = {0: "[PAD]", 100: "[UNK]", 101: "[CLS]", 102: "[SEP]", 103: "[MASK]"}
    vocab = [special.get(i, ch.get(i, f"[unused{i}]")) for i in range(BERT_BASE.vocab)]
    (tmp_path / "vocab.txt").write_text("\n".join(vocab) + "\n", encoding="utf-8")
    text = {}
    for u in range(nb.n_utt):
        for k, h in enumerate(range(nb.utt_off[u], nb.utt_off[u + 1])):
            text.setdefault(f"utt_{u}", {})[f"hyp_{k + 1}"] = "".join(ch[int(t)] for t in nb.hyp_words(h))
    json.dump(text, open(tmp_path / "hyps.json", "w", encoding="utf-8"), ensure_ascii=False)
    outs = {}
    for world in (1, 2):
        out = tmp_path / f"w{world}"
        out.mkdir()
        cfg = tmp_path / f"score_w{world}.yaml"
        cfg.write_text(yaml.safe_dump({
            "task": "scoring", "device": "cuda:0", "random_init_seed": 1234, "max_rows": 131072,
            "dev_hyps_text_path": str(tmp_path / "hyps.json"), "output_path": str(out) + "/",
            "model": {"bert": "bert-base-chinese", "vocab": str(tmp_path / "vocab.txt")}}, allow_unicode=True))
        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
        sk.close()
        code = ("import sys; sys.path.insert(0, %r); import __graft_entry__ as g; g._import_pkg(); "
                "from asr_rescoring_amd import cli; sys.exit(cli.main(['mlm_pll', '--config', %r]))" % (REPO, str(cfg)))
        procs = [subprocess.Popen([sys.executable, "-c", code],
                                  env=dict(os.environ, WORLD_SIZE=str(world), RANK=str(r), LOCAL_RANK="0",
                                           MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RS_DIST_BACKEND="gloo"))
                 for r in range(world)]
        for p in procs:
            assert p.wait(timeout=300) == 0
        outs[world] = json.load(open(out / "dev_lm.json", encoding="utf-8"))
    assert list(outs[1]) == list(outs[2]) == [f"utt_{u}" for u in range(nb.n_utt)]
    a = np.array([v for u in outs[1].values() for v in u.values()])
    b = np.array([v for u in outs[2].values() for v in u.values()])
    assert np.array_equal(a, b), np.abs(a - b).max()
    assert np.array_equal(a, pll), np.abs(a - pll).max()
