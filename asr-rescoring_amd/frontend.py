"""Native host front end: BertTokenizer-compatible tokenisation and the
score-JSON writer, in C++ behind the C-ABI (``csrc/tokenizer.cpp``, ``include/rescore.h``).

* ``NativeTokenizer(vocab_path)`` — ``tokenize``-free id interface of transformers'
  ``BertTokenizer(vocab_file, do_lower_case=True)`` as the reference uses it
  (``MLM_PLL/preprocess.py:9-30``, ``RescoreBert/preprocess.py:8-55``:
  ``convert_tokens_to_ids(tokenize(text))`` wrapped in [CLS] .. [SEP]);
  ``encode_nbest`` turns N-best texts straight into the ragged (tokens, hyp_off) layout of
  ``rs_pll_score`` / ``rs_cls_score``.
* ``json_saving(path, data)`` — ``util/saving.py:14-16`` (``json.dump(indent=4,
  ensure_ascii=False)``) for the {utt: {hyp: float}} score files, written natively.

Text is NFC-normalised here (``unicodedata.normalize``) before the native call; everything
after that (cleaning, CJK isolation, lower-casing, accent stripping, punctuation split,
WordPiece) runs in C++.  Known difference: Greek capital sigma is lower-cased without the
word-final rule of ``str.lower``.
"""
from __future__ import annotations

import ctypes
import unicodedata
from typing import Dict, List, Sequence, Tuple

import numpy as np

from . import _lib


class NativeTokenizer:
    def __init__(self, vocab_path: str):
        self.lib = _lib.load()
        self.handle = self.lib.rs_vocab_load(vocab_path.encode())
        if not self.handle:
            raise FileNotFoundError(f"cannot read vocab {vocab_path!r}")
        self.vocab_size = self.lib.rs_vocab_size(self.handle)

    def close(self):
        if getattr(self, "handle", None):
            self.lib.rs_vocab_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def encode_batch(self, texts: Sequence[str], add_special: bool = True) -> Tuple[np.ndarray, np.ndarray]:
        """(ids int32 [total], offsets int64 [n+1]) for n texts."""
        n = len(texts)
        arr = (ctypes.c_char_p * max(n, 1))(*[unicodedata.normalize("NFC", t).encode("utf-8") for t in texts])
        off = np.zeros(n + 1, np.int64)
        cap = max(64, sum(len(t) for t in texts) * 2 + 2 * n)
        while True:
            ids = np.empty(cap, np.int32)
            total = self.lib.rs_tokenize_batch(self.handle, arr, n, int(add_special), ids.ctypes.data, cap,
                                               off.ctypes.data)
            if total < 0:
                raise ValueError("rs_tokenize_batch: bad arguments")
            if total <= cap:
                return ids[:total].copy(), off
            cap = int(total)

    def encode(self, text: str, add_special: bool = False) -> List[int]:
        ids, _ = self.encode_batch([text], add_special)
        return ids.tolist()

    # interface used by cli.py (CharTokenizer-compatible)
    def encode_words(self, text: str) -> List[int]:
        return self.encode(text, add_special=False)

    def encode_nbest(self, hyps_text: Dict[str, Dict[str, str]], n_best: int = 1 << 30,
                     max_utt: int = 1 << 30):
        """N-best texts -> (tokens, hyp_off, utt_off, keys) in JSON key order."""
        texts, keys, uoff = [], [], [0]
        for u, (uid, hyps) in enumerate(hyps_text.items()):
            if u == max_utt:
                break
            for k, (hid, t) in enumerate(hyps.items()):
                if k == n_best:
                    break
                texts.append(t)
                keys.append((uid, hid))
            uoff.append(len(texts))
        ids, off = self.encode_batch(texts, add_special=True)
        return ids, off.astype(np.int32), np.asarray(uoff, np.int32), keys


def json_saving(path: str, data: Dict[str, Dict[str, float]]) -> None:
    """util/saving.py:14-16 for score files ({utt: {hyp: number}}), native writer; any other
    shape falls back to json.dump (same bytes)."""
    flat_ok = all(isinstance(v, dict) and all(isinstance(x, float) for x in v.values()) for v in data.values())
    if not flat_ok:
        import json
        with open(path, "w", encoding="utf8") as f:
            json.dump(data, f, ensure_ascii=False, indent=4)
        return
    utt = [u.encode("utf-8") for u in data]
    hyp_ids, scores, hoff = [], [], [0]
    for v in data.values():
        hyp_ids += [h.encode("utf-8") for h in v]
        scores += list(v.values())
        hoff.append(len(hyp_ids))
    lib = _lib.load()
    ua = (ctypes.c_char_p * max(len(utt), 1))(*utt)
    ha = (ctypes.c_char_p * max(len(hyp_ids), 1))(*hyp_ids)
    hoff_a = np.asarray(hoff, np.int32)
    sc = np.asarray(scores, np.float64)
    rc = lib.rs_json_write_scores(path.encode(), len(utt), ua, hoff_a.ctypes.data, ha, sc.ctypes.data)
    if rc != 0:
        raise OSError(f"cannot write {path!r}")
