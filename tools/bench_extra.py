"""Secondary measurements of the SURVEY §8d configurations (not the headline bench line).

  c2  RescoreBert: U=1000 x N=50 synthetic hypotheses -> CLS scores (fp16x3 default and fp16),
      hypothesis forwards/s and canonical TFLOP/s (5.425 GFLOP per forward at T=34).
  c4  MLM_PLL on the real-length variant (alfred test length histogram, N=100); a 1/10
      subsample of the 7176 test utterances (full C4 is ~10.5 M forwards).
  c5  RMBR CER utility: U=7176 x N=100 real-length hypotheses -> all-pairs edit distances
      (DP cells/s), MBR scores for k = 2..10, plus the 101-weight AM/LM fusion sweep.
  c5bs RMBR BERTScore utility at the C5 shape: 8-layer bert-base token embeddings + the
      all-pairs greedy-cosine recall matrix, MBR for k = 2..10.

Prints one JSON line per configuration.  usage: python tools/bench_extra.py [c2,c4,c5,c5bs]
"""
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__  # noqa: E402

__graft_entry__._import_pkg()
from asr_rescoring_amd import data as D  # noqa: E402
from asr_rescoring_amd import rerank  # noqa: E402
from asr_rescoring_amd.weights import BERT_BASE, make_weights  # noqa: E402


def _lengths():
    lc = json.load(open(os.path.join(REPO, "tests", "golden", "alfred_test_lengths.json")))["length_counts"]
    return np.repeat(np.arange(len(lc)), lc).astype(np.int64)


def _timed(fn, steps=2, warmup=1):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def rescorebert_flops(T, s=BERT_BASE):
    H, F, nl = s.hidden, s.intermediate, s.layers
    dense = 2 * (4 * H * H + 2 * H * F)
    return float((nl - 1) * (T * dense + 4 * T * T * H) + 4 * T * H * H
                 + (2 * H * H + 4 * T * H + 2 * H * H + 4 * H * F) + 2 * H)


def c2():
    from asr_rescoring_amd.scorer import RescoreBertScorer
    w = make_weights(BERT_BASE, seed=1234, with_cls_linear=True, with_pooler=True)
    nb = D.synthetic_nbest(1000, 50, seed=1)
    lens = np.diff(nb.hyp_off)
    fl = float(sum(rescorebert_flops(int(T)) for T in lens))
    d_tok = torch.from_numpy(nb.tokens).cuda()
    out = []
    for prec in ("fp16x3", "fp16"):
        sc = RescoreBertScorer(w, BERT_BASE, device=0, max_rows=131072, precision=prec)
        dt = _timed(lambda: sc.score_nbest(d_tok, nb.hyp_off))
        sc.profile(True)
        sc.score_nbest(d_tok, nb.hyp_off)
        torch.cuda.synchronize()
        kinds = sc.profile_read()
        sc.profile(False)
        sc.close()
        out.append({"workload": "C2 RescoreBert U=1000 N=50", "precision": prec, "value": round(nb.n_hyp / dt, 1),
                    "unit": "hypothesis fwd/s", "ms_per_step": round(dt * 1e3, 2),
                    "achieved_tflops_canonical": round(fl / dt / 1e12, 1),
                    "kinds_ms": {k: round(v[0], 2) for k, v in kinds.items()}})
    return out


def c4():
    from asr_rescoring_amd.scorer import PLLScorer
    w = make_weights(BERT_BASE, seed=1234)
    sc = PLLScorer(w, BERT_BASE, device=0, max_rows=131072)
    nb = D.synthetic_nbest(718, 100, seed=1, lengths=_lengths())
    d_tok = torch.from_numpy(nb.tokens).cuda()
    dt = _timed(lambda: sc.score_nbest(d_tok, nb.hyp_off), steps=1)
    prec = sc.precision
    sc.close()
    lens = np.diff(nb.hyp_off)
    return [{"workload": "C4 MLM_PLL real-length (718 of 7176 utts) N=100", "value": round(nb.n_forwards() / dt, 1),
             "unit": "masked fwd/s", "precision": prec,
             "dtype": "fp16x3-split (fp32-accurate)" if prec == "fp16x3" else "fp16 (reduced precision)",
             "parity": "tests/test_gpu_configs.py::test_c4_shape_real_lengths_mixed_chunk_and_ranks (rows/PLL vs oracle <1e-3, rerank argmax equal, 1 vs 2 ranks bitwise)",
             "forwards": nb.n_forwards(), "mean_T": round(float(np.average(lens, weights=lens - 2)), 2),
             "ms_per_step": round(dt * 1e3, 1)}]


def c5():
    nb = D.synthetic_nbest(7176, 100, seed=1, lengths=_lengths(), vocab=5000)
    lens = nb.hyp_len().astype(np.int64)
    cells = 0
    for u in range(nb.n_utt):
        l = lens[nb.utt_off[u]:nb.utt_off[u + 1]]
        s = int(l.sum())
        cells += s * s - int((l * l).sum())          # ordered pairs i != j
    holder = {}

    def pair():
        holder["ed"], holder["moff"] = rerank.pairwise_edit(nb, 0)
    dt_pair = _timed(pair)
    ed, moff = holder["ed"], holder["moff"]
    # kernel alone (inputs resident on the device, HIP events on the current stream)
    import ctypes
    from asr_rescoring_amd import _lib
    lib = _lib.load()
    flat, soff = rerank._strings(nb)
    d_c, d_so = torch.from_numpy(flat).cuda(), torch.from_numpy(soff).cuda()
    d_uo, d_mo = torch.from_numpy(np.ascontiguousarray(nb.utt_off, np.int32)).cuda(), torch.from_numpy(moff).cuda()
    st = torch.cuda.current_stream().cuda_stream
    kcall = lambda: _lib.check(lib.rs_pairwise_edit(_lib.ptr(d_c), _lib.ptr(d_so), _lib.ptr(d_uo), _lib.ptr(d_mo),
                                                    nb.n_utt, 100, _lib.ptr(ed), st))
    kcall()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        kcall()
    e1.record()
    torch.cuda.synchronize()
    dt_kern = e0.elapsed_time(e1) / 5 * 1e-3
    dt_mbr = _timed(lambda: [rerank.mbr_scores(nb, k, ed, moff, 0) for k in range(2, 11)])
    lm = -np.abs(np.random.default_rng(2).normal(40, 10, nb.n_hyp))
    grid = rerank.weight_grid("norm")
    am_d, lm_d = torch.from_numpy(nb.am).cuda(), torch.from_numpy(lm).cuda()
    dt_fuse = _timed(lambda: rerank.fuse_rerank(am_d, lm_d, nb.hyp_len(), nb.utt_off, grid, "norm", 100, 0))
    return [{"workload": "C5 RMBR CER utility U=7176 N=100 real-length", "value": round(cells / dt_pair / 1e9, 2),
             "value_note": "end to end incl. host flattening + H2D + 284 MB output allocation",
             "unit": "G DP cells/s (all ordered pairs)", "pairs": int(sum(int(n) * (int(n) - 1) for n in np.diff(nb.utt_off))),
             "ms_pairwise": round(dt_pair * 1e3, 2), "ms_pairwise_kernel": round(dt_kern * 1e3, 3),
             "kernel_G_cells_per_s": round(cells / dt_kern / 1e9, 1), "ms_mbr_k2_10": round(dt_mbr * 1e3, 2),
             "ms_fusion_sweep_101w": round(dt_fuse * 1e3, 2)}]


def c5bs():
    """BERTScore utility at the C5 shape: bert-base (8 of 12 layers, bert_score's truncation)
    embeddings of every hypothesis token + the greedy-cosine recall matrix of all ordered pairs."""
    from asr_rescoring_amd import bertscore as BS
    w = make_weights(BERT_BASE, seed=1234)
    nb = D.synthetic_nbest(7176, 100, seed=1, lengths=_lengths())
    sc = BS.BertScorer(w, BERT_BASE, num_layers=8, device=0, max_rows=131072)
    d_tok = torch.from_numpy(nb.tokens).cuda()
    rows = int(nb.hyp_off[-1])
    T = np.diff(nb.hyp_off).astype(np.int64)
    sT = np.add.reduceat(T, nb.utt_off[:-1]).astype(np.float64)
    H = BERT_BASE.hidden
    enc_fl = float(rows) * 8 * 2 * (4 * H * H + 2 * H * BERT_BASE.intermediate) + 8 * 4 * float((T * T).sum()) * H
    sim_fl = 2.0 * H * float((sT * sT).sum())
    dt_emb = _timed(lambda: sc.embed(d_tok, nb.hyp_off))
    holder = {}

    def rec():
        holder["r"] = sc.recall_matrix(d_tok, nb.hyp_off, nb.utt_off)
    dt_all = _timed(rec)
    rmat, moff = holder["r"]
    dt_mbr = _timed(lambda: [BS.mbr_scores(rmat, moff, nb.utt_off, k, "R") for k in range(2, 11)])
    sc.profile(True)
    sc.embed(d_tok, nb.hyp_off)
    torch.cuda.synchronize()
    kinds = {k: round(v[0], 1) for k, v in sc.profile_read().items()}
    sc.profile(False)
    sc.close()
    dt_sim = max(dt_all - dt_emb, 1e-9)
    return [{"workload": "C5 RMBR BERTScore utility U=7176 N=100 real-length, bert-base 8 layers",
             "value": round(int(moff[-1]) / dt_all / 1e6, 2), "unit": "M ordered pairs/s (embeddings included)",
             "tokens": rows, "ms_total": round(dt_all * 1e3, 1), "ms_embed": round(dt_emb * 1e3, 1),
             "ms_recall_kernel": round(dt_sim * 1e3, 1), "embed_tflops": round(enc_fl / dt_emb / 1e12, 1),
             "recall_tflops_algorithmic": round(sim_fl / dt_sim / 1e12, 1), "ms_mbr_k2_10": round(dt_mbr * 1e3, 2),
             "embed_ms_by_kind": kinds}]


def c2train():
    """RescoreBert distillation training (MD_MWER) on bert-base: batches of 3 utterances x
    N=50 (RescoreBert/main.py:75 batch_size * n_best rows), hypotheses / s and fp32 TFLOP/s
    (forward + backward ~ 3 x the forward's dense FLOPs)."""
    from asr_rescoring_amd.train import RescoreBertTrainer
    w = make_weights(BERT_BASE, seed=1234, with_cls_linear=True, with_pooler=True)
    tr = RescoreBertTrainer(w, BERT_BASE, method="MD_MWER", md_loss_weight=1e-4, lr=1e-5)  # MD_MWER_train.yaml
    nb = D.synthetic_nbest(3, 50, seed=1)
    rng = np.random.default_rng(0)
    tgt = -np.abs(rng.normal(40, 8, nb.n_hyp)).astype(np.float32)
    cer = (rng.integers(0, 6, nb.n_hyp) / 30.0).astype(np.float32)
    am = nb.am.astype(np.float32)
    step = lambda: tr.step(nb.tokens, nb.hyp_off, nb.utt_off, tgt, am, cer)
    dt = _timed(step, steps=5, warmup=2)
    tr.close()
    T = np.diff(nb.hyp_off).astype(np.float64)
    H, F, L = BERT_BASE.hidden, BERT_BASE.intermediate, BERT_BASE.layers
    fl = 3.0 * (float(T.sum()) * L * 2 * (4 * H * H + 2 * H * F) + L * 4 * float((T * T).sum()) * H)
    return [{"workload": "RescoreBert training MD_MWER, bert-base, 3 utts x N=50 per step (fp32)",
             "value": round(nb.n_hyp / dt, 1), "unit": "hypotheses/s", "rows_per_step": int(T.sum()),
             "ms_per_step": round(dt * 1e3, 1), "tflops_fp32": round(fl / dt / 1e12, 1)}]


def mlmtrain():
    """MLM fine-tuning on bert-base: the reference's batches (MLM_PLL/config/train.yaml: 32
    do_job rows, padded to the batch's longest, CE over every position) of reference-length
    sentences (L ~ U{24..40}); rows / s (one row = one masked copy) and fp32 TFLOP/s (3 x
    forward incl. the full-vocab head, over the padded positions the step computes)."""
    from asr_rescoring_amd.train import MLMTrainer, do_job_rows, pad_rows
    w = make_weights(BERT_BASE, seed=1234)
    tr = MLMTrainer(w, BERT_BASE, lr=1e-5)
    nb = D.synthetic_nbest(32, 1, seed=1)
    seqs = [nb.tokens[nb.hyp_off[h]:nb.hyp_off[h + 1]].tolist() for h in range(nb.n_hyp)]
    ids, off, lab = do_job_rows(seqs)
    rows = [ids[off[i]:off[i + 1]].tolist() for i in range(32)]
    labs = [lab[off[i]:off[i + 1]].tolist() for i in range(32)]
    batch = pad_rows(rows, labs)
    step = lambda: tr.step(*batch)
    dt = _timed(step, steps=5, warmup=2)
    tr.close()
    o = batch[1]
    T = np.diff(o).astype(np.float64)
    H, F, L, V = BERT_BASE.hidden, BERT_BASE.intermediate, BERT_BASE.layers, BERT_BASE.vocab
    fl = 3.0 * (float(T.sum()) * (L * 2 * (4 * H * H + 2 * H * F) + 2 * (H * H + H * V)) + L * 4 * float((T * T).sum()) * H)
    return [{"workload": "MLM fine-tuning, bert-base, 32 padded do_job rows per step (fp32)", "value": round(32 / dt, 1),
             "unit": "rows/s", "tokens_per_step": int(T.sum()), "ms_per_step": round(dt * 1e3, 1),
             "tflops_fp32": round(fl / dt / 1e12, 1)}]


def main():
    which = sys.argv[1].split(",") if len(sys.argv) > 1 else ["c2", "c4", "c5", "c5bs"]
    for name in which:
        for rec in {"c2": c2, "c4": c4, "c5": c5, "c5bs": c5bs, "c2train": c2train,
                    "mlmtrain": mlmtrain}[name]():
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
