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


if __name__ == "__main__":
    pytest.main([__file__, "-q"])
