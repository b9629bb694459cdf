"""Native front end (host-only, no GPU): tokenizer vs transformers.BertTokenizer on a local
vocab (the library the reference calls, run offline), JSON writer vs json.dump bytes."""
import json
import os
import random

import numpy as np
import pytest

from conftest import REPO  # noqa: F401

transformers = pytest.importorskip("transformers")

CJK = "你好嗎不是的我們今天天氣很好謝謝再見中文語音識別重新評分豈"
SPECIAL = ["[PAD]"] + [f"[unused{i}]" for i in range(1, 100)] + ["[UNK]", "[CLS]", "[SEP]", "[MASK]"]
WORDS = ["hello", "##llo", "he", "##l", "world", "##s", "the", "##re", "un", "##able", "play", "##ing",
         "cafe", "naive", "resume", "ab", "##c", "x", "##y", "1", "##2", "3", "i", "##i"]
PUNCT = list(",.!?;:'\"()[]{}-_/\\@#$%^&*+=<>~`|") + ["，", "。", "！", "？", "、", "「", "」", "—", "…"]


def _vocab(tmp_path):
    toks = SPECIAL + sorted(set(CJK)) + WORDS + PUNCT + ["豈"]
    p = tmp_path / "vocab.txt"
    p.write_text("\n".join(toks) + "\n", encoding="utf-8")
    return str(p)


def _random_text(rng: random.Random) -> str:
    pieces = []
    pool = (list(CJK) * 3 + WORDS[:3] + ["Hello", "WORLDS", "café", "naïve", "résumé", "ÀBC", "İi", "Straße",
            "playing", "unable", "xyz", "1234", "한국어", "日本語", "ＡＢＣ", "　", " ", "\t", "\n",
            "​", "\x07", "﻿", " ", "é", "[MASK]", "[CLS]", "[mask]", "x" * 120,
            "a" * 101, "🙂", "\U00020000", "豈",
            "\u2028", "\u2029", "\u0301", "e\u0301", "\u200b", "\u00a0", "\x85", "\u01c5", "\u216b",
            "\ufb01", "\uff76\uff9e"] + PUNCT)
    for _ in range(rng.randint(0, 25)):
        pieces.append(rng.choice(pool))
        if rng.random() < 0.4:
            pieces.append(" ")
    return "".join(pieces)


@pytest.fixture(scope="module")
def tok_pair(tmp_path_factory):
    from asr_rescoring_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("librescore.so not built")
    from asr_rescoring_amd.frontend import NativeTokenizer
    path = _vocab(tmp_path_factory.mktemp("vocab"))
    ref = transformers.BertTokenizer(path, do_lower_case=True)
    return NativeTokenizer(path), ref


def test_tokenizer_matches_bert_tokenizer_on_random_text(tok_pair):
    nat, ref = tok_pair
    rng = random.Random(0)
    texts = [_random_text(rng) for _ in range(1500)]
    ids, off = nat.encode_batch(texts, add_special=True)
    for i, t in enumerate(texts):
        want = [ref.cls_token_id] + ref.convert_tokens_to_ids(ref.tokenize(t)) + [ref.sep_token_id]
        got = ids[off[i]:off[i + 1]].tolist()
        assert got == want, (t, got, want)


def test_tokenizer_known_cases(tok_pair):
    nat, ref = tok_pair
    for t in ["你好嗎 Hello, worlds!", "", "   ", "[MASK]你好", "abc[MASK]def", "Naïve café", "　再見　"]:
        assert nat.encode(t) == ref.convert_tokens_to_ids(ref.tokenize(t)), t


def test_encode_nbest_layout(tok_pair):
    nat, _ = tok_pair
    hyps = {"u1": {"hyp_1": "你好", "hyp_2": "你好嗎"}, "u2": {"hyp_1": "再見"}}
    toks, hoff, uoff, keys = nat.encode_nbest(hyps)
    assert hoff.tolist() == [0, 4, 9, 13] and uoff.tolist() == [0, 2, 3]
    assert keys == [("u1", "hyp_1"), ("u1", "hyp_2"), ("u2", "hyp_1")]
    assert toks[0] == 101 and toks[3] == 102


def test_json_writer_is_byte_identical(tmp_path):
    from asr_rescoring_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("librescore.so not built")
    from asr_rescoring_amd.frontend import json_saving
    rng = np.random.default_rng(1)
    vals = [0.0, -0.0, 1.0, -1.5, 0.1, 1e-05, 0.0001, 123456789.0, 1e16, 1.2345678901234567e17, 1e-300,
            float("inf"), float("-inf"), float("nan"), 5e-324, 1.7976931348623157e308, -12.345]
    vals += list(rng.normal(0, 50, 200)) + list(-np.abs(rng.normal(0, 1, 50)) * 10.0 ** rng.integers(-8, 20, 50))
    data, k = {}, 0
    for u in range(20):
        uid = ["utt_中文", "a\"b\\c\n\t\x01", "plain", "é"][u % 4] + str(u)
        data[uid] = {}
        for h in range(rng.integers(0, 8)):
            data[uid][f"hyp_{h + 1}"] = float(vals[k % len(vals)])
            k += 1
    a, b = tmp_path / "a.json", tmp_path / "b.json"
    json_saving(str(a), data)
    with open(b, "w", encoding="utf8") as f:
        json.dump(data, f, ensure_ascii=False, indent=4)
    assert a.read_bytes() == b.read_bytes()
    json_saving(str(a), {})
    assert a.read_bytes() == b"{}"
