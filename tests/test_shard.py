"""Multi-rank path on CPU (gloo, world_size 2): sharding plan + the one all-gather of (am, lm)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from asr_rescoring_amd import data as D
from asr_rescoring_amd.shard import gather_scores, plan_shards, utterance_costs


def test_plan_shards_balanced_and_contiguous():
    nb = D.synthetic_nbest(37, 7, seed=3, len_lo=2, len_hi=60)
    c = utterance_costs(nb)
    for world in (1, 2, 3, 8):
        parts = plan_shards(c, world)
        assert parts[0][0] == 0 and parts[-1][1] == nb.n_utt
        assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
        loads = [c[a:b].sum() for a, b in parts]
        assert max(loads) - min(loads) <= 2 * c.max()


def test_plan_shards_more_ranks_than_utts():
    parts = plan_shards([5.0, 1.0], 4)
    assert sum(b - a for a, b in parts) == 2 and parts[-1][1] == 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    nb = D.synthetic_nbest(9, 5, seed=11)
    parts = plan_shards(utterance_costs(nb), world)
    u0, u1 = parts[rank]
    h0, h1 = nb.utt_off[u0], nb.utt_off[u1]
    # stand-in "lm" = a deterministic function of the hypothesis tokens (the GPU scorer's
    # role); the test checks the exchange, not the scores
    lm = np.array([float(nb.tokens[nb.hyp_off[h]:nb.hyp_off[h + 1]].sum()) for h in range(h0, h1)])
    local = torch.stack([torch.from_numpy(nb.am[h0:h1]), torch.from_numpy(lm)])
    counts = [int(nb.utt_off[b] - nb.utt_off[a]) for a, b in parts]
    out = gather_scores(local, counts)
    if rank == 0:
        q.put(out.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_gather_matches_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    nb = D.synthetic_nbest(9, 5, seed=11)
    lm = np.array([float(nb.tokens[nb.hyp_off[h]:nb.hyp_off[h + 1]].sum()) for h in range(nb.n_hyp)])
    assert np.array_equal(got[0], nb.am)
    assert np.array_equal(got[1], lm)


def test_exchange_device_rules():
    from asr_rescoring_amd.shard import exchange_device
    assert exchange_device("gloo", torch.device("cpu")) == torch.device("cpu")
    assert exchange_device("gloo", torch.device("cpu"), "cuda:0") == torch.device("cpu")
    assert exchange_device(None, torch.device("cpu")) == torch.device("cpu")
    assert exchange_device("nccl", torch.device("cpu"), "cuda:1") == torch.device("cuda", 1)
    if torch.cuda.is_available():
        # an empty shard's CPU placeholder goes to this rank's GPU under RCCL
        assert exchange_device("nccl", torch.device("cpu")).type == "cuda"


def _tok_sum_fn(sub):
    return torch.tensor([float(sub.tokens[sub.hyp_off[h]:sub.hyp_off[h + 1]].sum()) for h in range(sub.n_hyp)],
                        dtype=torch.float64)


def _worker_empty(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from asr_rescoring_amd.shard import score_sharded
    nb = D.synthetic_nbest(1, 6, seed=13)          # one utterance, two ranks: rank 1 owns nothing
    calls = []
    both = score_sharded(nb, lambda sub: (calls.append(sub.n_utt), _tok_sum_fn(sub))[1])
    q.put((rank, both.numpy(), calls))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_empty_shard():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_empty, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict((r, (b, c)) for r, b, c in (q.get(timeout=120), q.get(timeout=120)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    nb = D.synthetic_nbest(1, 6, seed=13)
    want = np.stack([nb.am, _tok_sum_fn(nb).numpy()])
    # one rank owns the utterance, the other none and never calls the scorer
    assert sorted([got[0][1], got[1][1]]) == [[], [1]]
    for r in (0, 1):
        assert np.array_equal(got[r][0], want)


def _oracle_pll_fn(model):
    """Per-hypothesis oracle PLL (CPU fp32, batch = one hypothesis' rows): independent of how
    utterances are split, so sharded and single-process scores must be bitwise equal."""
    from oracle.bert_ref import pll_reference_pattern

    def fn(sub):
        out = []
        for h in range(sub.n_hyp):
            toks = sub.tokens[sub.hyp_off[h]:sub.hyp_off[h + 1]]
            out.append(pll_reference_pattern(model, toks, np.array([0, len(toks)]), batch_size=64,
                                             full_head=False)[1][0])
        return torch.tensor(out, dtype=torch.float64)
    return fn


class _OracleRowScorer:
    """Stand-in for PLLScorer.row_logprobs on CPU (oracle masked_logprob_ref per row)."""
    device = torch.device("cpu")

    def __init__(self, model):
        self.model = model

    def row_logprobs(self, rows):
        from oracle.bert_ref import masked_logprob_ref
        out = [masked_logprob_ref(self.model, np.asarray([r["input_ids"]]), np.ones((1, len(r["input_ids"]))),
                                  np.asarray([r["labels"]]), np.asarray([r["mask_pos"]]))[0] for r in rows]
        return torch.tensor(out, dtype=torch.float32)


def _tiny_case():
    from asr_rescoring_amd.weights import BERT_TINY, make_weights
    from oracle.bert_ref import TorchBert
    torch.set_num_threads(1)
    nb = D.synthetic_nbest(5, 4, seed=12, vocab=BERT_TINY.vocab, len_lo=2, len_hi=9, hard=True)
    return nb, TorchBert(make_weights(BERT_TINY, seed=7), BERT_TINY)


def _rows_of(nb):
    from oracle.bert_ref import pll_rows
    rows = []
    for h, ids, mp, lab in pll_rows(nb.tokens, nb.hyp_off):
        u = int(np.searchsorted(nb.utt_off, h, side="right") - 1)
        rows.append({"utt_id": f"u{u}", "hyp_id": f"hyp_{h - nb.utt_off[u] + 1}", "input_ids": ids,
                     "mask_pos": mp, "labels": lab})
    return rows


def _worker_score(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK="0", RS_DIST_BACKEND="gloo")
    from asr_rescoring_amd import cli
    from asr_rescoring_amd.shard import init_from_env, score_sharded
    from oracle import rescore_ref as RR
    init_from_env()
    nb, model = _tiny_case()
    both = score_sharded(nb, _oracle_pll_fn(model))
    rows_out = cli._score_rows_sharded(_OracleRowScorer(model), _rows_of(nb), rank, world)
    if rank == 0:
        N = 4
        hyps = [[nb.hyp_words(nb.utt_off[u] + i) for i in range(N)] for u in range(nb.n_utt)]
        lm = both[1].numpy().reshape(nb.n_utt, N)
        fused = RR.find_best_weight(both[0].numpy().reshape(nb.n_utt, N), lm, hyps, nb.refs, n_best=N)
        q.put((both.numpy(), fused[0], fused[1], fused[2], rows_out))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_score_gather_fuse_bitwise():
    """Split -> score (oracle PLL as the scorer) -> one all-gather -> rank-0 fusion sweep
    (rescore.py:25-45), and the do_job-rows path of ``cli mlm_pll`` on 2 ranks: bitwise equal
    to the single-process results."""
    from asr_rescoring_amd import cli
    from oracle import rescore_ref as RR
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_score, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got, bw, bcer, arg, rows_out = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    nb, model = _tiny_case()
    lm = _oracle_pll_fn(model)(nb).numpy()
    assert np.array_equal(got[0], nb.am) and np.array_equal(got[1], lm)
    N = 4
    hyps = [[nb.hyp_words(nb.utt_off[u] + i) for i in range(N)] for u in range(nb.n_utt)]
    bw1, bcer1, arg1 = RR.find_best_weight(nb.am.reshape(nb.n_utt, N), lm.reshape(nb.n_utt, N), hyps, nb.refs,
                                           n_best=N)
    assert bw == bw1 and bcer == bcer1 and np.array_equal(arg, arg1)
    assert rows_out == cli._score_rows_sharded(_OracleRowScorer(model), _rows_of(nb), 0, 1)


if __name__ == "__main__":
    pytest.main([__file__, "-q"])
