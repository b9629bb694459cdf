"""GPU: robustness of the fused residual + LayerNorm GEMM (EPI_LNRES_IMG) and of the call
contract around it, plus the RCCL exchange on one GPU.

* gangs (the column tiles of a row panel exchanging row statistics inside the launch) are formed
  by start-order tickets (per XCD by default, RS_LNGANG=xcd; chip-wide with RS_LNGANG=ticket) and
  claim their row panels: with most CUs held by another process's kernel the call scores beside it,
  bitwise equal to an idle GPU; with whole shader engines held it is delayed like any kernel, not
  failed;
* the timeout path itself (forced by a diagnostic bit): RS_EHIP with a message, the flag cleared,
  the next call clean;
* the chip-wide ticket form (RS_LNGANG=ticket) scores bitwise like the XCD-local default;
* chunks cut at whole LayerNorm-gang rounds score bitwise like max_rows chunks;
* the deferred range check (rs_model_set_sync_check / rs_check);
* a one-rank ``nccl`` (RCCL) process group: ``shard.score_sharded`` / ``gather_scores`` /
  ``cli._score_rows_sharded`` on device tensors, bitwise equal to the undistributed path.
"""
import ctypes
import os

import numpy as np
import pytest
import torch

from asr_rescoring_amd import _lib
from asr_rescoring_amd import data as D
from asr_rescoring_amd.weights import BERT_BASE, BERT_TINY, make_weights

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def w_base():
    return make_weights(BERT_BASE, seed=1234)


@pytest.fixture(scope="module")
def nb_mid():
    # ~20k token rows per layer: 86+ row panels, several tiles per workgroup in every launch
    return D.synthetic_nbest(12, 20, seed=21, vocab=BERT_BASE.vocab, len_lo=10, len_hi=40)


@pytest.fixture(scope="module")
def scorer(w_base):
    from asr_rescoring_amd.scorer import PLLScorer
    s = PLLScorer(w_base, BERT_BASE, device=0, max_rows=32768, precision="fp16x3")
    yield s
    s.close()


@pytest.fixture(scope="module")
def base_scores(scorer, nb_mid):
    return scorer.score(nb_mid)


_OCCUPIER = r"""
import ctypes, sys, time
import torch
sys.path.insert(0, {repo!r})
import __graft_entry__
__graft_entry__._import_pkg()
from asr_rescoring_amd import _lib
lib = _lib.load()
fn = lib.rs_debug_occupy
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
out = torch.zeros(4096, dtype=torch.int32, device="cuda")
torch.cuda.synchronize()
assert fn({blocks}, {usec}, out.data_ptr(), torch.cuda.current_stream().cuda_stream) == 0
time.sleep(0.05)
print("ready", flush=True)
torch.cuda.synchronize()
t_end = time.time()
print("done", int(out[:{blocks}].min().item()), repr(t_end), flush=True)
"""


class _Occupier:
    """Another PROCESS holding `blocks` CUs (one 160 KiB-LDS workgroup each) for `usec` us.  In one
    process the occupying kernel and the scorer's kernels shared a hardware queue (GPU_MAX_HW_QUEUES
    = 4) or the null stream's implicit synchronisation, and the call simply ran after the occupier
    (3.0 s = the occupier's 3 s; the round-4 form of these tests never shared the GPU)."""

    def __init__(self, blocks, usec):
        import subprocess
        import sys
        repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        code = _OCCUPIER.format(repo=repo, blocks=blocks, usec=usec)
        self.p = subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE, text=True)
        line = self.p.stdout.readline().strip()
        assert line == "ready", line

    def wait(self):
        """The occupier's output; ``self.t_end``: wall time (time.time()) its kernel was seen done."""
        out = self.p.stdout.read()
        assert self.p.wait(timeout=60) == 0, out
        self.t_end = float(out.split()[-1])
        return out


def _n_cu():
    return torch.cuda.get_device_properties(0).multi_processor_count


@pytest.mark.parametrize("gang", ["xcd", "ticket"])
@pytest.mark.parametrize("free", ["quarter", "one_per_engine"])
def test_lnfuse_scores_beside_another_process(scorer, nb_mid, base_scores, monkeypatch, gang, free):
    """Another process's kernel holds three quarters of the CUs, or all but one CU of each of the 32
    shader engines (one 160 KiB-LDS workgroup each), for 3 s while the scorer runs: the gangs form
    from whichever workgroups start and claim every row panel between them (nb_mid has ~86 panels
    per launch, far more than the gangs that fit), the call returns long before the occupier ends,
    and the scores are bitwise those of an idle GPU.  (Before round 5 each gang owned a fixed set of
    panels, so a launch needed all of its workgroups to start.)"""
    import time
    monkeypatch.setenv("RS_LNGANG", gang)
    held = _n_cu() * 3 // 4 if free == "quarter" else _n_cu() - 32
    occ = _Occupier(held, 3_000_000)
    t0 = time.perf_counter()
    got = scorer.score(nb_mid)
    t_ret = time.time()
    dt = time.perf_counter() - t0
    occ.wait()
    print(f"scored beside {held} held CUs in {dt:.2f} s ({gang}); occupier ended {occ.t_end - t_ret:.2f} s later")
    # the call returned while the occupier still held its CUs (no wall-clock bound of our own: the
    # occupier's end is the reference, whatever the box's speed)
    assert t_ret < occ.t_end, f"the call waited for the occupier ({dt:.2f} s)"
    assert np.array_equal(got, base_scores)


def test_lnfuse_full_engines_delay_but_do_not_fail(scorer, nb_mid, base_scores):
    """All but 8 CUs held by another process for 1.5 s: some shader engines are full, and the
    workgroups the hardware dispatches to them wait for a free CU there (every kernel's do —
    tools/diag/occupy_probe3.py: a 1-ms kernel or a library GEMM then takes the occupier's time).
    The call is delayed, not failed: no statistics wait runs out, and the scores are bitwise."""
    import time
    occ = _Occupier(_n_cu() - 8, 1_500_000)
    t0 = time.perf_counter()
    got = scorer.score(nb_mid)
    dt = time.perf_counter() - t0
    occ.wait()
    print(f"scored with full shader engines in {dt:.2f} s")
    assert np.array_equal(got, base_scores)


def test_lnfuse_forced_timeout_reports_and_clears(scorer, nb_mid, base_scores, monkeypatch):
    """RS_LNFUSE_DIAG=8 makes every statistics and gang wait time out at once: the call fails
    with RS_EHIP and says so; the sticky flag is cleared, so the next call scores cleanly."""
    from asr_rescoring_amd._lib import RescoreError
    monkeypatch.setenv("RS_LNFUSE_DIAG", "8")
    with pytest.raises(RescoreError, match="timed out waiting for its row statistics"):
        scorer.score(nb_mid)
    monkeypatch.delenv("RS_LNFUSE_DIAG")
    assert np.array_equal(scorer.score(nb_mid), base_scores)


def test_lnfuse_ticket_gangs_match_xcd_gangs(scorer, nb_mid, base_scores, monkeypatch):
    """The chip-wide ticket form computes every tile with the same statistics order as the
    XCD-local default: bitwise equal scores."""
    monkeypatch.setenv("RS_LNGANG", "ticket")
    assert np.array_equal(scorer.score(nb_mid), base_scores)


@pytest.fixture(scope="module")
def nb_small():
    return D.synthetic_nbest(2, 6, seed=23, vocab=BERT_BASE.vocab, len_lo=10, len_hi=24)


def test_chunks_at_gang_rounds_match(w_base, nb_mid, monkeypatch):
    """run_all cuts chunks at multiples of 256 x (LayerNorm gangs) rows (RS_CHUNK_ALIGN, default
    on); rows are computed independently of their chunk, so the scores are bitwise those of
    plain max_rows chunks."""
    from asr_rescoring_amd.scorer import PLLScorer
    s = PLLScorer(w_base, BERT_BASE, device=0, max_rows=24000, precision="fp16x3")
    try:
        a = s.score(nb_mid)
        monkeypatch.setenv("RS_CHUNK_ALIGN", "0")
        b = s.score(nb_mid)
    finally:
        s.close()
    assert np.array_equal(a, b)


def test_calls_on_two_streams_are_ordered(scorer, nb_mid, nb_small, base_scores):
    """Calls on one handle issued on two streams without any synchronisation between them (the
    deferred mode, so the calls return at once): the handle orders them (a call on another stream
    waits for the previous call's event), so both results equal the single-stream scores."""
    base_small = scorer.score(nb_small)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    scorer.set_sync_check(False)
    try:
        with torch.cuda.stream(s1):
            a = scorer.score_nbest(torch.from_numpy(nb_mid.tokens).cuda(), nb_mid.hyp_off)
        with torch.cuda.stream(s2):
            b = scorer.score_nbest(torch.from_numpy(nb_small.tokens).cuda(), nb_small.hyp_off)
        with torch.cuda.stream(s1):
            c = scorer.score_nbest(torch.from_numpy(nb_mid.tokens).cuda(), nb_mid.hyp_off)
        with torch.cuda.stream(s2):
            scorer.check()
        torch.cuda.synchronize()
    finally:
        scorer.set_sync_check(True)
    assert np.array_equal(a.cpu().numpy(), base_scores)
    assert np.array_equal(b.cpu().numpy(), base_small)
    assert np.array_equal(c.cpu().numpy(), base_scores)


def test_deferred_range_check():
    """rs_model_set_sync_check(0): an overflowing call returns without synchronising; rs_check
    reports RS_EUNSUP once and clears it; synchronous mode restored."""
    from asr_rescoring_amd._lib import RescoreError
    from asr_rescoring_amd.scorer import PLLScorer
    w = make_weights(BERT_TINY, seed=7)
    g = "bert.embeddings.LayerNorm.weight"
    w_bad = dict(w)
    w_bad[g] = w[g] * 1e6
    nb = D.synthetic_nbest(2, 3, seed=5, vocab=BERT_TINY.vocab, len_lo=3, len_hi=12)
    s = PLLScorer(w_bad, BERT_TINY, device=0, max_rows=2048)
    try:
        s.set_sync_check(False)
        s.score_nbest(nb.tokens, nb.hyp_off)            # no exception: deferred
        s.score_nbest(nb.tokens, nb.hyp_off)
        with pytest.raises(RescoreError, match="non-finite"):
            s.check()
        s.check()                                        # cleared
        s.set_sync_check(True)
        with pytest.raises(RescoreError, match="non-finite"):
            s.score_nbest(nb.tokens, nb.hyp_off)
    finally:
        s.close()
    ok = PLLScorer(w, BERT_TINY, device=0, max_rows=2048)
    try:
        ok.set_sync_check(False)
        a = ok.score_nbest(nb.tokens, nb.hyp_off)
        ok.check()
        ok.set_sync_check(True)
        assert np.array_equal(a.cpu().numpy(), ok.score(nb))
    finally:
        ok.close()


def test_rccl_exchange_one_rank(w_base, monkeypatch):
    """A one-rank ``nccl`` (RCCL) process group, as ``shard.init_from_env(force=True)`` makes it:
    score_sharded's all_gather_into_tensor runs on device tensors and returns the (am, lm) block
    bitwise equal to the undistributed path; cli._score_rows_sharded takes the gather branch;
    an empty N-best list (no local utterance) keeps the block on this rank's GPU."""
    import torch.distributed as dist
    from asr_rescoring_amd import cli, shard
    from asr_rescoring_amd.scorer import PLLScorer
    nb = D.synthetic_nbest(6, 10, seed=3, vocab=BERT_BASE.vocab, len_lo=6, len_hi=20)
    s = PLLScorer(w_base, BERT_BASE, device=0, max_rows=8192, precision="fp16x3")
    assert not dist.is_initialized()
    fn = lambda sub: s.score_nbest(sub.tokens, sub.hyp_off)       # noqa: E731
    plain = shard.score_sharded(nb, fn)
    rows = []
    for u in range(nb.n_utt):
        for k, h in enumerate(range(nb.utt_off[u], nb.utt_off[u + 1])):
            seq = nb.tokens[nb.hyp_off[h]:nb.hyp_off[h + 1]].tolist()
            for p in range(1, len(seq) - 1):
                ids = list(seq)
                ids[p] = BERT_BASE.mask_id
                rows.append({"utt_id": f"u{u}", "hyp_id": f"hyp_{k + 1}", "input_ids": ids, "labels": seq,
                             "mask_pos": p})
    plain_rows = cli._score_rows_sharded(s, rows, 0, 1)
    monkeypatch.delenv("RS_DIST_BACKEND", raising=False)
    for k, v in (("RANK", "0"), ("WORLD_SIZE", "1"), ("LOCAL_RANK", "0"), ("MASTER_ADDR", "127.0.0.1"),
                 ("MASTER_PORT", str(29600 + os.getpid() % 300))):
        monkeypatch.setenv(k, v)
    try:
        rank, world, local = shard.init_from_env(force=True)
        assert (rank, world) == (0, 1) and dist.is_initialized() and dist.get_backend() == "nccl"
        both = shard.score_sharded(nb, fn)
        assert both.device.type == "cuda"
        assert torch.equal(both.cpu(), plain.cpu())
        got_rows = cli._score_rows_sharded(s, rows, 0, 1)
        assert got_rows == plain_rows
        empty = shard.score_sharded(nb.slice_utts(0, 0), fn)
        assert tuple(empty.shape) == (2, 0) and empty.device.type == "cuda"
        g = shard.gather_scores(both, [both.shape[1]])
        assert torch.equal(g, both)
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()
        s.close()
