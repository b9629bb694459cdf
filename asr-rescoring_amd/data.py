"""N-best lists as ragged token arrays, synthetic generators and the score-JSON format.

Layout (what the C-ABI consumes, see ``include/rescore.h``):

* ``tokens``  int32 [sum_h T_h] — every hypothesis as ``[CLS] w_1 .. w_L [SEP]``,
  exactly the ``labels`` row of ``MLM_PLL/preprocess.py:24-28`` and the
  ``hyps_token_ids`` row of ``RescoreBert/preprocess.py:32-39``.
* ``hyp_off`` int32 [H+1] — hypothesis h owns ``tokens[hyp_off[h]:hyp_off[h+1]]``.
* ``utt_off`` int32 [U+1] — utterance u owns hypotheses ``utt_off[u]:utt_off[u+1]``.

Synthetic inputs follow SURVEY §8d (PCG64 seeded): per utterance a base sentence of
L0 ~ U{24..40} ids drawn from [106, V); each hypothesis applies k ~ U{0..3} random
substitutions / insertions / deletions; AM scores are sorted-descending -|N(5.8, 4)|.
"""
from __future__ import annotations

import dataclasses
import json
from typing import Dict, List, Optional, Sequence

import numpy as np

CLS_ID, SEP_ID, MASK_ID, PAD_ID, UNK_ID = 101, 102, 103, 0, 100
FIRST_WORD_ID = 106


@dataclasses.dataclass
class NBest:
    tokens: np.ndarray          # int32 [sum T]
    hyp_off: np.ndarray         # int32 [H+1]
    utt_off: np.ndarray         # int32 [U+1]
    am: np.ndarray              # float64 [H]
    refs: List[np.ndarray]      # per utterance int32 reference ids (no CLS/SEP)
    utt_ids: List[str]
    hyp_ids: List[str]
    lens: Optional[np.ndarray] = None   # per-hypothesis len(text) when built from text

    @property
    def n_hyp(self) -> int:
        return len(self.hyp_off) - 1

    @property
    def n_utt(self) -> int:
        return len(self.utt_off) - 1

    def hyp_len(self) -> np.ndarray:
        """Length in words/characters (T - 2); ``rescore.py:28-35`` uses ``len(hyp)``."""
        if self.lens is not None:
            return np.asarray(self.lens, np.int32)
        return (np.diff(self.hyp_off) - 2).astype(np.int32)

    def hyp_words(self, h: int) -> np.ndarray:
        return self.tokens[self.hyp_off[h] + 1:self.hyp_off[h + 1] - 1]

    def n_forwards(self) -> int:
        """Number of masked forwards R = sum_h L_h (one per masked position)."""
        return int(self.hyp_len().sum())

    def slice_utts(self, u0: int, u1: int) -> "NBest":
        """Contiguous utterance range [u0, u1) (vectorised; a rank's shard)."""
        h0, h1 = int(self.utt_off[u0]), int(self.utt_off[u1])
        t0, t1 = int(self.hyp_off[h0]), int(self.hyp_off[h1])
        return NBest(np.ascontiguousarray(self.tokens[t0:t1], np.int32),
                     (np.asarray(self.hyp_off[h0:h1 + 1], np.int64) - t0).astype(np.int32),
                     (np.asarray(self.utt_off[u0:u1 + 1], np.int64) - h0).astype(np.int32),
                     np.asarray(self.am[h0:h1], np.float64), list(self.refs[u0:u1]),
                     list(self.utt_ids[u0:u1]), list(self.hyp_ids[h0:h1]))

    def subset(self, utts: Sequence[int]) -> "NBest":
        toks, hoff, uoff, am, hyp_ids, refs, uids = [], [0], [0], [], [], [], []
        for u in utts:
            for h in range(self.utt_off[u], self.utt_off[u + 1]):
                seg = self.tokens[self.hyp_off[h]:self.hyp_off[h + 1]]
                toks.append(seg)
                hoff.append(hoff[-1] + len(seg))
                am.append(self.am[h])
                hyp_ids.append(self.hyp_ids[h])
            uoff.append(len(hoff) - 1)
            refs.append(self.refs[u])
            uids.append(self.utt_ids[u])
        return NBest(np.concatenate(toks).astype(np.int32) if toks else np.zeros(0, np.int32),
                     np.asarray(hoff, np.int32), np.asarray(uoff, np.int32),
                     np.asarray(am, np.float64), refs, uids, hyp_ids)


def from_lists(hyps: List[List[Sequence[int]]], am: Optional[List[List[float]]] = None,
               refs: Optional[List[Sequence[int]]] = None,
               utt_ids: Optional[List[str]] = None) -> NBest:
    """Build an ``NBest`` from per-utterance lists of word-id lists (no CLS/SEP)."""
    toks, hoff, uoff, amv, hyp_ids = [], [0], [0], [], []
    for u, utt in enumerate(hyps):
        for k, w in enumerate(utt):
            seq = [CLS_ID] + [int(x) for x in w] + [SEP_ID]
            toks.extend(seq)
            hoff.append(hoff[-1] + len(seq))
            amv.append(float(am[u][k]) if am is not None else 0.0)
            hyp_ids.append(f"hyp_{k + 1}")
        uoff.append(len(hoff) - 1)
    uids = utt_ids or [f"utt_{u}" for u in range(len(hyps))]
    rf = [np.asarray(r, np.int32) for r in refs] if refs is not None else \
         [np.asarray(h[0], np.int32) for h in hyps]
    return NBest(np.asarray(toks, np.int32), np.asarray(hoff, np.int32),
                 np.asarray(uoff, np.int32), np.asarray(amv, np.float64), rf, uids, hyp_ids)


def from_texts(hyps_text: Dict[str, Dict[str, str]], ref_text: Optional[Dict[str, str]] = None,
               am: Optional[Dict[str, Dict[str, float]]] = None, n_best: int = 1 << 30,
               max_utt: int = 1 << 30) -> NBest:
    """N-best of raw strings for the CER side (jiwer semantics): symbols are the characters
    of ``text.strip()`` (Unicode code points), ``lens`` keeps ``len(text)`` as
    ``rescore.py:28-35`` computes it.  JSON key order defines utterance / hypothesis order
    (``rescore.py:13-23`` relies on it too)."""
    words, ams, refs, uids, lens = [], [], [], [], []
    for u, (uid, hyps) in enumerate(hyps_text.items()):
        if u == max_utt:
            break
        items = list(hyps.items())[:n_best]
        words.append([[ord(c) for c in t.strip()] for _, t in items])
        lens.extend(len(t) for _, t in items)
        ams.append([float(am[uid][h]) for h, _ in items] if am is not None else [0.0] * len(items))
        refs.append([ord(c) for c in ref_text[uid].strip()] if ref_text is not None else [])
        uids.append(uid)
    nb = from_lists(words, ams, refs, uids)
    nb.hyp_ids = [h for uid in uids for h in list(hyps_text[uid])[:n_best]]
    nb.lens = np.asarray(lens, np.int32)
    return nb


def _edit(rng: np.random.Generator, base: List[int], k: int, vocab: int) -> List[int]:
    w = list(base)
    for _ in range(k):
        op = int(rng.integers(0, 3))
        if op == 0 and w:                       # substitution
            w[int(rng.integers(0, len(w)))] = int(rng.integers(FIRST_WORD_ID, vocab))
        elif op == 1:                           # insertion
            w.insert(int(rng.integers(0, len(w) + 1)), int(rng.integers(FIRST_WORD_ID, vocab)))
        elif len(w) > 1:                        # deletion (never empty)
            del w[int(rng.integers(0, len(w)))]
    return w


def synthetic_nbest(n_utt: int, n_best: int, seed: int = 1, vocab: int = 21128,
                    len_lo: int = 24, len_hi: int = 40, max_edits: int = 3,
                    lengths: Optional[np.ndarray] = None, hard: bool = False) -> NBest:
    """Seeded synthetic N-best lists.

    ``lengths`` (optional) is a histogram sample of base lengths (real-length variant).
    Hypotheses within an utterance are distinct where possible (like ESPnet beams).
    ``hard``: the reference-identical hypothesis is not first and the AM scores are not
    sorted (hypotheses permuted, AM drawn per hypothesis), so the fused argmax moves with the
    weight and the reranked CER is not simply the AM-only CER (parity tests of the rerank).
    """
    rng = np.random.Generator(np.random.PCG64(seed))
    hyps, ams, refs = [], [], []
    for _ in range(n_utt):
        L0 = int(rng.choice(lengths)) if lengths is not None else int(rng.integers(len_lo, len_hi + 1))
        base = [int(x) for x in rng.integers(FIRST_WORD_ID, vocab, size=L0)]
        seen, utt = set(), []
        for k in range(n_best):
            for _attempt in range(8):
                w = _edit(rng, base, int(rng.integers(0, max_edits + 1)) if k else 0, vocab)
                if tuple(w) not in seen:
                    break
            seen.add(tuple(w))
            utt.append(w)
        am = -np.abs(rng.normal(5.8, 4.0, size=n_best))
        if hard:
            perm = rng.permutation(n_best)
            utt = [utt[int(i)] for i in perm]
            ams.append(am.tolist())
        else:
            ams.append(np.sort(am)[::-1].tolist())
        hyps.append(utt)
        refs.append(base)
    return from_lists(hyps, ams, refs)


# ---------------------------------------------------------------------------------------
# Score JSON format: {utt_id: {hyp_id: float}}  (util/saving.py:14-16, indent 4,
# ensure_ascii False; skeleton from util/get_output_format.py:4-16).
# ---------------------------------------------------------------------------------------

def scores_to_json_dict(nb: NBest, scores: np.ndarray) -> Dict[str, Dict[str, float]]:
    out: Dict[str, Dict[str, float]] = {}
    for u, uid in enumerate(nb.utt_ids):
        row = {}
        for h in range(nb.utt_off[u], nb.utt_off[u + 1]):
            row[nb.hyp_ids[h]] = float(scores[h])
        out[uid] = row
    return out


def json_saving(path: str, data) -> None:
    """Byte-compatible with ``util/saving.py:14-16``."""
    with open(path, "w", encoding="utf8") as f:
        json.dump(data, f, ensure_ascii=False, indent=4)


def get_output_format(path: str, max_utt: int, n_best: int) -> Dict[str, Dict[str, float]]:
    """Mirror of ``util/get_output_format.py:4-16`` (skeleton of zeros)."""
    origin = json.load(open(path, "r", encoding="utf-8"))
    out: Dict[str, Dict[str, float]] = {}
    for u, (uid, hyps) in enumerate(origin.items()):
        if u == max_utt:
            break
        out[uid] = {}
        if isinstance(hyps, dict):
            for k, hid in enumerate(hyps):
                if k == n_best:
                    break
                out[uid][hid] = 0
    return out


class CharTokenizer:
    """Char-level stand-in for ``BertTokenizer`` on CJK text (which splits CJK per char).

    No ``vocab.txt`` exists offline, so ids are assigned from a char list:
    [PAD]=0, [UNK]=100, [CLS]=101, [SEP]=102, [MASK]=103, chars from 106 upward.
    """

    def __init__(self, chars: Sequence[str]):
        self.vocab = {c: FIRST_WORD_ID + i for i, c in enumerate(sorted(set(chars)))}

    def tokenize(self, text: str) -> List[str]:
        return [c for c in text.strip() if not c.isspace()]

    def convert_tokens_to_ids(self, toks: Sequence[str]) -> List[int]:
        special = {"[CLS]": CLS_ID, "[SEP]": SEP_ID, "[MASK]": MASK_ID, "[PAD]": PAD_ID}
        return [special.get(t, self.vocab.get(t, UNK_ID)) for t in toks]

    def encode_words(self, text: str) -> List[int]:
        return self.convert_tokens_to_ids(self.tokenize(text))
