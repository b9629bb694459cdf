"""Trainer GEMM picker (k_sgemm.hip sg_pick / sg_model), host only: the tile configuration and
split-K count chosen for the bert-base training shapes on MI355X's 256 CUs are the measured-best
ones (profiles/r3u_sgemm_pick.txt), and the choice is a function of the shape and the CU count
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


def test_192x128_where_the_128x128_grid_leaves_a_half_round(pick):
    # 5300 x 2304 x 768 forward: 756 tiles of 128x128 = 1.48 rounds; 504 tiles of 192x128 = 1
    assert pick(5300, 2304, 768) == (9, 1)
    # 5300 x 3072 x 768: 1008 tiles of 128x128 = 2 full rounds -> 128x128, no split
    assert pick(5300, 3072, 768) == (0, 1)


def test_small_batches_64x64_direct_or_split_k(pick):
    # 1100 x 768 x 768: 54 tiles of 128x128 need split-K; 216 tiles of the 64x64 direct form fill
    # the chip in one pass (27.5 -> 18.7 us, profiles/r4f_sgemm_cfg11.txt)
    assert pick(1100, 768, 768) == (11, 1)
    assert pick(2304, 768, 1100, 1) == (11, 1)  # a ~1k-token weight gradient (55.1 -> 44.9 us)
    cfg, sp = pick(768, 768, 5300, 1)           # weight gradient over 5.3k tokens
    assert cfg == 0 and sp > 1


def test_choice_is_a_function_of_shape_and_cus(pick):
    shapes = [(1100, 2304, 768, 0), (2304, 768, 1100, 1), (5300, 768, 3072, 0)]
    a = [pick(m, n, k, f) for m, n, k, f in shapes]
    b = [pick(m, n, k, f) for m, n, k, f in shapes]
    assert a == b
    # a device with fewer CUs rounds differently: 756 tiles of 128x128 on 128 CUs x 2 = 2.95
    # rounds, against 1.48 on 256 CUs where the 192x128 tile's single round wins
    assert pick(5300, 2304, 768, 0, 256) == (9, 1)
    assert pick(5300, 2304, 768, 0, 0) == (-1, 99)        # rejected
