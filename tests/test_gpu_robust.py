"""GPU: robustness of the fused residual + LayerNorm GEMM (EPI_LNRES_IMG) and of the call
contract around it, plus the RCCL exchange on one GPU.

* gangs (the column tiles of a row panel exchanging row statistics inside the launch) are formed
  by start-order tickets (per XCD by default, RS_LNGANG=xcd; chip-wide with RS_LNGANG=ticket): with
  most CUs held by another stream's kernel the call still scores, bitwise equal to an idle GPU,
  and never reaches the statistics-wait timeout;
* the timeout path itself (forced by a diagnostic bit): RS_EHIP with a message, the flag cleared,
  the next call clean;
* the chip-wide ticket form (RS_LNGANG=ticket) scores bitwise like the XCD-local default;
* the co-residency limit stated in include/rescore.h: with only two free workgroup slots (bert-base
  gangs need three) the call fails fast with RS_EHIP instead of hanging, and the next call on a free
  GPU scores bitwise (the gang-ticket words are reset by every launch); with three free slots the
  ticket form scores;
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


def _occupy(blocks, usec, stream):
    lib = _lib.load()
    fn = lib.rs_debug_occupy
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    assert fn(blocks, usec, None, stream.cuda_stream) == 0


def test_lnfuse_scores_with_cus_held_by_another_stream(scorer, nb_mid, base_scores):
    """Another stream's kernel holds 240 of the CUs (one 160 KiB-LDS workgroup each) for 0.3 s
    while the scorer runs: the ticket gangs form from whichever workgroups start, the launch
    completes on the CUs left, the scores are bitwise those of an idle GPU."""
    side = torch.cuda.Stream()
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    _occupy(max(1, n_cu - 16), 300_000, side)
    got = scorer.score(nb_mid)
    torch.cuda.synchronize()
    assert np.array_equal(got, base_scores)


def test_lnfuse_forced_timeout_reports_and_clears(scorer, nb_mid, base_scores, monkeypatch):
    """RS_LNFUSE_DIAG=8 makes every statistics wait time out at once: the call fails with
    RS_EHIP and says so; the sticky flag is cleared, so the next call scores cleanly."""
    from asr_rescoring_amd._lib import RescoreError
    monkeypatch.setenv("RS_LNFUSE_DIAG", "8")
    with pytest.raises(RescoreError, match="timed out waiting for its row statistics"):
        scorer.score(nb_mid)
    monkeypatch.delenv("RS_LNFUSE_DIAG")
    assert np.array_equal(scorer.score(nb_mid), base_scores)


def test_lnfuse_ticket_gangs_match_xcd_gangs(scorer, nb_mid, base_scores, monkeypatch):
    """The chip-wide ticket form computes the same tiles with the same statistics order as the
    XCD-local default: bitwise equal scores, also with CUs held elsewhere."""
    monkeypatch.setenv("RS_LNGANG", "ticket")
    assert np.array_equal(scorer.score(nb_mid), base_scores)
    side = torch.cuda.Stream()
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    _occupy(n_cu // 2, 300_000, side)
    got = scorer.score(nb_mid)
    torch.cuda.synchronize()
    assert np.array_equal(got, base_scores)


@pytest.fixture(scope="module")
def nb_small():
    # one launch chunk, ~3k token rows: the kernels around the LayerNorm GEMMs stay short on 2-3 CUs
    return D.synthetic_nbest(2, 6, seed=23, vocab=BERT_BASE.vocab, len_lo=10, len_hi=24)


@pytest.mark.parametrize("gang", ["ticket", "xcd"])
def test_lnfuse_too_few_free_slots_fails_fast_then_recovers(scorer, nb_small, monkeypatch, gang):
    """Another stream's kernel holds all but two CUs (one 160 KiB-LDS workgroup each) for 4 s: a
    bert-base gang (three column tiles) can never be co-resident, the first statistics wait runs
    out, every other wait sees the error word and gives up, and the call fails with RS_EHIP well
    before the CUs free up.  Once they have, the next call scores bitwise like an idle GPU."""
    import time
    from asr_rescoring_amd._lib import RescoreError
    monkeypatch.setenv("RS_LNGANG", gang)
    base = scorer.score(nb_small)
    side = torch.cuda.Stream()
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    _occupy(n_cu - 2, 4_000_000, side)
    t0 = time.perf_counter()
    with pytest.raises(RescoreError, match="timed out"):
        scorer.score(nb_small)
    dt = time.perf_counter() - t0
    side.synchronize()
    print(f"RS_EHIP after {dt:.2f} s with 2 free CUs ({gang})")
    assert dt < 3.5, dt
    assert np.array_equal(scorer.score(nb_small), base)


def test_lnfuse_three_free_slots_suffice(scorer, nb_small, monkeypatch):
    """All but three CUs held: the ticket gangs (three start-order tickets anywhere) still form and
    the call scores bitwise like an idle GPU."""
    monkeypatch.setenv("RS_LNGANG", "ticket")
    base = scorer.score(nb_small)
    side = torch.cuda.Stream()
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    _occupy(n_cu - 3, 2_000_000, side)
    got = scorer.score(nb_small)
    torch.cuda.synchronize()
    assert np.array_equal(got, base)


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
