"""Utterance sharding across ranks + the one RCCL exchange of the rescoring job.

The reference is single-process (``config.device``, MLM_PLL/main.py:187,
RescoreBert/main.py:252).  Utterances are independent, so rank r scores a contiguous range
of utterances chosen to balance cost (MLM_PLL: sum_h L_h * (L_h + 2) token rows;
RescoreBert: sum_h T_h), and the only collective is one ``all_gather_into_tensor`` of the
(am, lm) score block so that the fusion/rerank step (rescore.py) sees every hypothesis.
Contiguous ranges keep global order: the gather needs no permutation.  One process per GPU;
backend "nccl" (= RCCL over xGMI on ROCm), or "gloo" for the CPU tests.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from .data import NBest


def utterance_costs(nb: NBest, mode: str = "pll") -> np.ndarray:
    T = np.diff(nb.hyp_off).astype(np.int64)
    per_hyp = (T - 2) * T if mode == "pll" else T
    return np.add.reduceat(per_hyp, nb.utt_off[:-1]) if nb.n_utt else np.zeros(0, np.int64)


def plan_shards(costs: Sequence[float], world: int) -> List[Tuple[int, int]]:
    """Contiguous [u0, u1) ranges, one per rank, greedy on the cost prefix sum."""
    c = np.asarray(costs, np.float64)
    n = len(c)
    if world <= 1:
        return [(0, n)]
    pref = np.concatenate([[0.0], np.cumsum(c)])
    total = pref[-1]
    cuts = [0]
    for r in range(1, world):
        target = total * r / world
        k = int(np.searchsorted(pref, target, side="left"))
        # choose the closer of k-1 / k, never going backwards
        if k > 0 and abs(pref[k - 1] - target) <= abs(pref[min(k, n)] - target):
            k -= 1
        cuts.append(max(cuts[-1], min(k, n)))
    cuts.append(n)
    return [(cuts[i], cuts[i + 1]) for i in range(world)]


def gather_scores(local: torch.Tensor, counts: Sequence[int], group=None) -> torch.Tensor:
    """all_gather of a [C, n_local] block (C score columns, e.g. am and lm) padded to the
    largest shard; returns the [C, sum(counts)] concatenation in rank order."""
    world = dist.get_world_size(group)
    C = local.shape[0]
    width = max(counts)
    buf = torch.zeros(C, width, dtype=local.dtype, device=local.device)
    buf[:, :local.shape[1]] = local
    out = torch.empty(world * C, width, dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, buf.reshape(-1, width).contiguous(), group=group)
    out = out.view(world, C, width)
    return torch.cat([out[r, :, :counts[r]] for r in range(world)], dim=1)


def init_from_env(device_index: int | None = None, force: bool = False):
    """torchrun / torch.distributed.run launch: (rank, world, local_rank).  Initialises the
    default process group once (backend "nccl" = RCCL when a GPU is visible, else "gloo") when
    WORLD_SIZE > 1, or at any world size with ``force`` (a one-rank group: the exchange code
    path runs unchanged on one GPU; MASTER_ADDR / MASTER_PORT default to 127.0.0.1:29512)."""
    import os
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0")) if device_index is None else device_index
    # RS_DIST_BACKEND=gloo: CPU exchange (e.g. several ranks sharing one GPU in a test)
    backend = os.environ.get("RS_DIST_BACKEND", "nccl" if torch.cuda.is_available() else "gloo")
    if force and world == 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29512")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    if (world > 1 or force) and not dist.is_initialized():
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    return rank, world, local


def shard_of(nb: NBest, world: int, rank: int, mode: str = "pll") -> Tuple[int, int]:
    """This rank's contiguous utterance range [u0, u1) (cost-balanced, ``plan_shards``)."""
    return plan_shards(utterance_costs(nb, mode), world)[rank]


def exchange_device(backend, lm_device, device=None) -> torch.device:
    """Where the (am, lm) block must live for the all-gather: CPU under gloo; under nccl
    (RCCL) always this rank's GPU — also on a rank whose shard is empty, where the scorer
    never ran and there is no device tensor to take it from (an empty CPU block would make
    RCCL raise or hang the group)."""
    if backend == "gloo":
        return torch.device("cpu")
    if device is not None:
        return torch.device(device)
    if backend is not None:
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device(lm_device)


def score_sharded(nb: NBest, score_fn, mode: str = "pll", device=None, group=None) -> torch.Tensor:
    """Utterance-sharded scoring with one all-gather (MLM_PLL/main.py:164-203 on
    N ranks).  ``score_fn(sub_nbest) -> lm [H_local]`` scores this rank's utterances (the HIP
    scorer in the product; any callable in tests).  Returns the (am, lm) float64 block
    [2, H] of EVERY hypothesis, in global order, on every rank.  A rank may own no
    utterance (fewer utterances than ranks, or a few costly ones taking the prefix sum)."""
    distributed = dist.is_initialized()
    world = dist.get_world_size(group) if distributed else 1
    rank = dist.get_rank(group) if distributed else 0
    parts = plan_shards(utterance_costs(nb, mode), world)
    u0, u1 = parts[rank]
    sub = nb.slice_utts(u0, u1)
    h0, h1 = int(nb.utt_off[u0]), int(nb.utt_off[u1])
    lm = score_fn(sub) if h1 > h0 else torch.zeros(0, dtype=torch.float64)
    lm = torch.as_tensor(lm).to(torch.float64)
    dev = exchange_device(dist.get_backend(group) if distributed else None, lm.device, device)
    am = torch.from_numpy(np.ascontiguousarray(nb.am[h0:h1], np.float64)).to(dev)
    local = torch.stack([am, lm.to(dev)])
    if not distributed:            # with a process group (also of one rank) the exchange runs
        return local
    counts = [int(nb.utt_off[b] - nb.utt_off[a]) for a, b in parts]
    if max(counts) == 0:
        return local
    return gather_scores(local, counts, group)
