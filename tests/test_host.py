"""Host-side checks without a GPU: the C-ABI library loads and exports every declared symbol."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import REPO


def declared_symbols():
    src = open(os.path.join(REPO, "include", "rescore.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rs_[a-z_0-9]+)\s*\(", src)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ("rs_model_create", "rs_model_set_tensor", "rs_model_finalize", "rs_pll_score",
              "rs_masked_logprob", "rs_cls_score", "rs_pairwise_edit", "rs_mbr_scores",
              "rs_fuse_rerank", "rs_corpus_edits", "rs_ref_edit", "rs_last_error", "rs_model_destroy"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from asr_rescoring_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("librescore.so not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for s in declared_symbols():
        assert hasattr(lib, s), s
    # the ctypes signature table covers the header
    assert set(declared_symbols()) <= set(_lib.EXPORTED)
    loaded = _lib.load()
    assert loaded.rs_version() >= 1
    assert isinstance(loaded.rs_last_error(), bytes)


def test_create_without_gpu_fails_cleanly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from asr_rescoring_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("librescore.so not built")
    lib = _lib.load()
    cfg = _lib.RsBertCfg(1000, 256, 2, 4, 1024, 512, 2, 1e-12, 103, 1, 0)
    h = ctypes.c_void_p()
    rc = lib.rs_model_create(ctypes.byref(cfg), 0, ctypes.byref(h))
    assert rc != 0 and b"device" in lib.rs_last_error()


def test_scorer_refuses_cpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from asr_rescoring_amd.scorer import PLLScorer
    from asr_rescoring_amd.weights import BERT_TINY, make_weights
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        PLLScorer(make_weights(BERT_TINY), BERT_TINY)


def test_config_yaml_roundtrip(tmp_path):
    from asr_rescoring_amd.config import parse_config, load_yaml
    p = tmp_path / "c.yaml"
    p.write_text("task: scoring\nseed: 10\ndataloader:\n  batch_size: 32\n  num_worker: 5\nmodel:\n  bert: x\n")
    c = parse_config(load_yaml(str(p)))
    assert c.task == "scoring" and c.dataloader.batch_size == 32 and c.model.bert == "x"
    _ = np


def test_attention_mask_validation():
    """RescoreBertHIP.forward / masked_logprob accept only right-padded 0/1 masks."""
    import torch
    from asr_rescoring_amd.scorer import _prefix_lengths
    ok = torch.tensor([[1, 1, 1, 0], [1, 1, 1, 1], [1, 0, 0, 0]])
    assert _prefix_lengths(ok).tolist() == [3, 4, 1]
    for bad in ([[0, 1, 1, 1]], [[1, 0, 1, 0]], [[1, 2, 0, 0]]):
        with pytest.raises(ValueError):
            _prefix_lengths(torch.tensor(bad))
