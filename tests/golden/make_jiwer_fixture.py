"""jiwer CER golden vectors from a data file the reference holds (this container only).

Run from the repo root:  ``python tests/golden/make_jiwer_fixture.py``  (needs /root/reference).

``/root/reference/Nbest_Align/cer.json`` is a list of 7176 ``{"ref", "pred", "cer"}`` records:
a reference transcript, a predicted sentence and the CER that ``jiwer.cer`` gave for the pair
(``Nbest_Align/preprocess.py:8,132`` is the reference's call site of the same function).  jiwer
is absent from this image, so these recorded outputs are the only jiwer results
available: they pin the CER restatement (oracle) and the CER kernels (``rs_ref_edit``) at the
jiwer boundary.

Written: ``tests/golden/jiwer_cer_pairs.json`` = {"source", "pairs": [[ref, pred, cer], ...]}
with every record whose CER is non-zero (the ones that exercise the edit distance) plus the
first 200 zero-CER records — data only (inputs and jiwer's outputs), no reference source.
"""
from __future__ import annotations

import json
import os

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = "/root/reference/Nbest_Align/cer.json"
OUT = os.path.join(REPO, "tests", "golden", "jiwer_cer_pairs.json")


def main() -> None:
    with open(SRC, encoding="utf-8") as f:
        recs = json.load(f)
    nz = [r for r in recs if r["cer"] != 0]
    zero = [r for r in recs if r["cer"] == 0][:200]
    pairs = [[r["ref"], r["pred"], r["cer"]] for r in nz + zero]
    with open(OUT, "w", encoding="utf-8") as f:
        json.dump({"source": "Nbest_Align/cer.json (jiwer.cer outputs recorded by the reference)",
                   "records_in_source": len(recs), "pairs": pairs}, f, ensure_ascii=False, indent=0)
    print(f"{len(pairs)} pairs ({len(nz)} non-zero CER) -> {OUT}")


if __name__ == "__main__":
    main()
