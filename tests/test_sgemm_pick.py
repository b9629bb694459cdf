"""Trainer GEMM picker (k_sgemm.hip sg_pick / sg_model), host only: the tile configuration and
split-K count chosen for the bert-base training shapes on MI355X's 256 CUs are the measured-best
ones (profiles/r6y_sgemm_split_sweep.txt), and the choice is a function of the shape and the CU count
(bitwise-reproducible training on a given device model).  The CU count is passed explicitly, so
these tests make no GPU call."""
import ctypes

import pytest

from asr_rescoring_amd import _lib


@pytest.fixture(scope="module")
def pick():
    lib = _lib.load()
    fn = lib.rs_debug_sgemm_pick
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int] * 5
    return lambda M, N, K, mcmc=0, cus=256: divmod(fn(M, N, K, mcmc, cus), 100)


def test_software_pipelined_tile_without_split_at_5k_tokens(pick):
    # 5300 x 2304 x 768 forward: 756 tiles of 128x128 on 256 CUs, no split (142 us measured; the
    # software-pipelined tile retires a K-step as fast alone on a CU as beside a second workgroup)
    assert pick(5300, 2304, 768) == (12, 1)
    assert pick(5300, 3072, 768) == (12, 1)
    # 252 tiles, 96 K-steps: one workgroup per CU, no split (183 us; split 2: 191 us)
    assert pick(5300, 768, 3072) == (12, 1)


def test_small_batches_64x64_direct_half_tiles_or_split_k(pick):
    # 1100 x 768 x 768: 54 tiles of 128x128; 216 tiles of the 64x64 direct form fill the chip in
    # one pass (18.7 us against 26.3 us for the 128x128 tile split 4 ways, 21.5 for 64x128 split 2)
    assert pick(1100, 768, 768) == (11, 1)
    # a ~1k-token weight gradient: 216 software-pipelined 64x128 tiles, one pass, no split
    # (40.8 us against 48.0 for the 128x128 tile split 2 ways, profiles/r6ab_sgemm_all.jsonl)
    assert pick(2304, 768, 1100, 1) == (17, 1)
    cfg, sp = pick(768, 768, 5300, 1)           # weight gradient over 5.3k tokens
    assert cfg == 12 and sp > 1
    # splits stop at two workgroups per CU (a third short round measured well above the model)
    cfg, sp = pick(1100, 768, 21128)            # the tied decoder's input gradient: 54 tiles
    assert cfg == 12 and 54 * sp <= 512


def test_choice_is_a_function_of_shape_and_cus(pick):
    shapes = [(1100, 2304, 768, 0), (2304, 768, 1100, 1), (5300, 768, 3072, 0)]
    a = [pick(m, n, k, f) for m, n, k, f in shapes]
    b = [pick(m, n, k, f) for m, n, k, f in shapes]
    assert a == b
    # a device with fewer CUs rounds differently: on 128 CUs the 64x64 direct form's 216 tiles
    # need two passes and the 108 software-pipelined 64x128 tiles fill the chip in one
    assert pick(1100, 768, 768, 0, 256) == (11, 1)
    assert pick(1100, 768, 768, 0, 128) == (17, 1)
    assert pick(5300, 2304, 768, 0, 0) == (-1, 99)        # rejected
