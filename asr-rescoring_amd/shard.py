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
