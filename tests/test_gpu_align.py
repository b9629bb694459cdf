"""GPU parity of the alignment kernel (rs_align, csrc/k_align.hip) with the oracle
restatement of espnet_data/preprocess/align.py:5-97 (oracle/align_ref.py): the reference's
known answers (align.py:12-18), random CJK pairs over small alphabets (so S / I / D cost ties
are frequent), empty sides, hypotheses longer than one 64-row strip, one launch per batch."""
import numpy as np
import pytest

from oracle.align_ref import levenshtein_distance_alignment as ref_align

pytestmark = pytest.mark.gpu

KNOWN = [
    (["how", "are", "you"], ["how", "are", "you", "doing"],
     [["how", "are", "you", "*"], ["how", "are", "you", "doing"], ["U", "U", "U", "D"]]),
    (list("你好嗎"), list("你好不好"), [["你", "好", "*", "嗎"], ["你", "好", "不", "好"], ["U", "U", "D", "S"]]),
]


def test_known_answers():
    from asr_rescoring_amd.align import align_batch, levenshtein_distance_alignment
    for r, h, want in KNOWN:
        assert levenshtein_distance_alignment(r, h) == want
    assert align_batch([(r, h) for r, h, _ in KNOWN]) == [w for *_, w in KNOWN]


def _rand_pairs(rng, n, lo, hi, alpha):
    chars = [chr(0x4e00 + k) for k in range(alpha)]
    pick = lambda: [chars[int(c)] for c in rng.integers(0, alpha, int(rng.integers(lo, hi + 1)))]  # noqa: E731
    return [(pick(), pick()) for _ in range(n)]


def test_random_pairs_match_oracle():
    from asr_rescoring_amd.align import align_batch
    rng = np.random.default_rng(0)
    pairs = _rand_pairs(rng, 400, 0, 20, 3) + _rand_pairs(rng, 200, 5, 40, 12)
    # N-best style: edits of one reference
    for _ in range(200):
        r = [chr(0x4e00 + int(c)) for c in rng.integers(0, 50, int(rng.integers(3, 30)))]
        h = list(r)
        for _ in range(int(rng.integers(0, 5))):
            k = int(rng.integers(0, 3))
            pos = int(rng.integers(0, len(h) + 1))
            if k == 0 and h:
                h[min(pos, len(h) - 1)] = chr(0x4e00 + int(rng.integers(0, 50)))
            elif k == 1:
                h.insert(pos, chr(0x4e00 + int(rng.integers(0, 50))))
            elif h:
                del h[min(pos, len(h) - 1)]
        pairs.append((r, h))
    got = align_batch(pairs)
    ties = 0
    for (r, h), g in zip(pairs, got):
        want = ref_align(r, h)
        assert g == want, (r, h, g, want)
        ties += sum(o != "U" for o in want[2])
    assert ties > 1000


def test_empty_and_long():
    from asr_rescoring_amd.align import align_batch
    rng = np.random.default_rng(1)
    long_pairs = _rand_pairs(rng, 3, 150, 300, 4) + [(list("ab" * 300), list("ba" * 280))]
    pairs = [([], []), (list("abc"), []), ([], list("xy"))] + long_pairs
    got = align_batch(pairs)
    assert got[0] == [[], [], []]
    assert got[1] == [list("abc"), ["*"] * 3, ["I"] * 3]
    assert got[2] == [["*"] * 2, list("xy"), ["D"] * 2]
    for (r, h), g in zip(long_pairs, got[3:]):
        assert g == ref_align(r, h)
