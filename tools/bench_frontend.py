"""Host front-end throughput: native tokenizer vs transformers.BertTokenizer (the library the
reference calls) on C4-like N-best texts, and the native score-JSON writer vs json.dump.
usage: python tools/bench_frontend.py [n_texts]"""
import json
import os
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__  # noqa: E402

__graft_entry__._import_pkg()
from asr_rescoring_amd.frontend import NativeTokenizer, json_saving  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
    rng = np.random.default_rng(0)
    chars = [chr(c) for c in range(0x4E00, 0x4E00 + 3000)]
    d = tempfile.mkdtemp()
    vocab = os.path.join(d, "vocab.txt")
    toks = ["[PAD]"] + [f"[unused{i}]" for i in range(1, 100)] + ["[UNK]", "[CLS]", "[SEP]", "[MASK]"] + chars
    open(vocab, "w", encoding="utf-8").write("\n".join(toks) + "\n")
    lens = rng.integers(5, 30, n)
    texts = ["".join(rng.choice(chars, L)) for L in lens]
    nat = NativeTokenizer(vocab)
    t0 = time.perf_counter()
    ids, off = nat.encode_batch(texts)
    t_nat = time.perf_counter() - t0
    rec = {"texts": n, "mean_chars": float(lens.mean()), "native_texts_per_s": round(n / t_nat)}
    try:
        from transformers import BertTokenizer
        ref = BertTokenizer(vocab, do_lower_case=True)
        m = min(n, 20000)
        t0 = time.perf_counter()
        for t in texts[:m]:
            ref.convert_tokens_to_ids(ref.tokenize(t))
        rec["transformers_texts_per_s"] = round(m / (time.perf_counter() - t0))
    except ImportError:
        pass
    data = {f"utt_{u}": {f"hyp_{h + 1}": float(v) for h, v in enumerate(rng.normal(-40, 10, 100))}
            for u in range(max(1, n // 100))}
    p1, p2 = os.path.join(d, "a.json"), os.path.join(d, "b.json")
    t0 = time.perf_counter()
    json_saving(p1, data)
    rec["native_json_scores_per_s"] = round(n / (time.perf_counter() - t0))
    t0 = time.perf_counter()
    with open(p2, "w", encoding="utf8") as f:
        json.dump(data, f, ensure_ascii=False, indent=4)
    rec["json_dump_scores_per_s"] = round(n / (time.perf_counter() - t0))
    rec["json_identical"] = open(p1, "rb").read() == open(p2, "rb").read()
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
