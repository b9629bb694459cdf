"""Deterministic BERT weights for the rescorer (no checkpoint download exists offline).

The reference loads ``bert-base-chinese`` by name (``MLM_PLL/main.py:184``,
``RescoreBert/model.py:7``) and then a fine-tuned ``state_dict`` via ``torch.load``
(``MLM_PLL/main.py:185-186``, ``RescoreBert/main.py:250-251``).  Neither exists in this
image, so every test, the golden fixtures and the benchmark use weights drawn from a
numpy PCG64 generator (seed 1234, std 0.05, LayerNorm gamma = 1 + N(0, 0.02),
beta = N(0, 0.02)).  Keys are the HuggingFace ``state_dict`` names, so a real checkpoint
in HF layout is a drop-in replacement (``load_state_dict_file``).
"""
from __future__ import annotations

import dataclasses
import hashlib
from typing import Dict, Iterator, Tuple

import numpy as np


@dataclasses.dataclass(frozen=True)
class BertShape:
    """Architecture hyper-parameters (``transformers.BertConfig`` field meanings)."""

    vocab: int = 21128          # bert-base-chinese vocabulary
    hidden: int = 768
    layers: int = 12
    heads: int = 12
    intermediate: int = 3072
    max_pos: int = 512
    type_vocab: int = 2
    ln_eps: float = 1e-12
    pad_id: int = 0
    unk_id: int = 100
    cls_id: int = 101
    sep_id: int = 102
    mask_id: int = 103

    @property
    def head_dim(self) -> int:
        return self.hidden // self.heads


BERT_BASE = BertShape()
# A small shape used by the fast kernel tests (same head_dim=64 as BERT-base).
BERT_TINY = BertShape(vocab=1000, hidden=256, layers=2, heads=4, intermediate=1024)


def mlm_keys(shape: BertShape, with_mlm_head: bool = True,
             with_cls_linear: bool = False, with_pooler: bool = False
             ) -> Iterator[Tuple[str, Tuple[int, ...], str]]:
    """Yield ``(hf_key, shape, kind)`` in generation order.

    kind: 'mat' (N(0, std)), 'bias' (N(0, 0.02)), 'ln_w' (1 + N(0, 0.02)), 'ln_b'.
    Key names follow ``BertForMaskedLM.state_dict()`` (MLM_PLL) and ``RescoreBert``
    (``RescoreBert/model.py:7-11``: ``bert.*`` + ``linear.weight``/``linear.bias``).
    """
    H, F, V = shape.hidden, shape.intermediate, shape.vocab
    e = "bert.embeddings."
    yield e + "word_embeddings.weight", (V, H), "mat"
    yield e + "position_embeddings.weight", (shape.max_pos, H), "mat"
    yield e + "token_type_embeddings.weight", (shape.type_vocab, H), "mat"
    yield e + "LayerNorm.weight", (H,), "ln_w"
    yield e + "LayerNorm.bias", (H,), "ln_b"
    for i in range(shape.layers):
        p = f"bert.encoder.layer.{i}."
        for name in ("query", "key", "value"):
            yield p + f"attention.self.{name}.weight", (H, H), "mat"
            yield p + f"attention.self.{name}.bias", (H,), "bias"
        yield p + "attention.output.dense.weight", (H, H), "mat"
        yield p + "attention.output.dense.bias", (H,), "bias"
        yield p + "attention.output.LayerNorm.weight", (H,), "ln_w"
        yield p + "attention.output.LayerNorm.bias", (H,), "ln_b"
        yield p + "intermediate.dense.weight", (F, H), "mat"
        yield p + "intermediate.dense.bias", (F,), "bias"
        yield p + "output.dense.weight", (H, F), "mat"
        yield p + "output.dense.bias", (H,), "bias"
        yield p + "output.LayerNorm.weight", (H,), "ln_w"
        yield p + "output.LayerNorm.bias", (H,), "ln_b"
    # Heads come last, in a fixed order, and are always drawn (then filtered by the flags)
    # so that a given seed yields the same tensor for a given key whatever heads are kept.
    c = "cls.predictions."
    heads = [(c + "transform.dense.weight", (H, H), "mat", with_mlm_head),
             (c + "transform.dense.bias", (H,), "bias", with_mlm_head),
             (c + "transform.LayerNorm.weight", (H,), "ln_w", with_mlm_head),
             (c + "transform.LayerNorm.bias", (H,), "ln_b", with_mlm_head),
             (c + "bias", (V,), "bias", with_mlm_head),
             ("bert.pooler.dense.weight", (H, H), "mat", with_pooler),
             ("bert.pooler.dense.bias", (H,), "bias", with_pooler),
             ("linear.weight", (1, H), "mat", with_cls_linear),
             ("linear.bias", (1,), "bias", with_cls_linear)]
    for key, shp, kind, keep in heads:
        yield key, shp, kind + ("" if keep else ":skip")


def make_weights(shape: BertShape = BERT_BASE, seed: int = 1234, std: float = 0.05,
                 with_mlm_head: bool = True, with_cls_linear: bool = False,
                 with_pooler: bool = False) -> Dict[str, np.ndarray]:
    """Seeded fp32 weights keyed by HF state_dict names.

    The MLM decoder is tied to the word embeddings (transformers
    ``BertForMaskedLM._tied_weights_keys``), so ``cls.predictions.decoder.weight`` is the
    same array as ``bert.embeddings.word_embeddings.weight`` and ``decoder.bias`` is
    ``cls.predictions.bias``.
    """
    rng = np.random.Generator(np.random.PCG64(seed))
    out: Dict[str, np.ndarray] = {}
    for key, shp, kind in mlm_keys(shape, with_mlm_head, with_cls_linear, with_pooler):
        n = int(np.prod(shp))
        z = rng.standard_normal(n, dtype=np.float32).reshape(shp)
        if kind.endswith(":skip"):
            continue
        if kind == "mat":
            z *= np.float32(std)
        elif kind in ("bias", "ln_b"):
            z *= np.float32(0.02)
        elif kind == "ln_w":
            z = np.float32(1.0) + np.float32(0.02) * z
        out[key] = np.ascontiguousarray(z, dtype=np.float32)
    if with_mlm_head:
        out["cls.predictions.decoder.weight"] = out["bert.embeddings.word_embeddings.weight"]
        out["cls.predictions.decoder.bias"] = out["cls.predictions.bias"]
    return out


def weights_digest(weights: Dict[str, np.ndarray]) -> str:
    """sha256 over sorted (key, bytes); recorded in the golden fixtures."""
    h = hashlib.sha256()
    for k in sorted(weights):
        h.update(k.encode())
        h.update(np.ascontiguousarray(weights[k], dtype=np.float32).tobytes())
    return h.hexdigest()


def load_state_dict_file(path: str) -> Dict[str, np.ndarray]:
    """Load a real checkpoint without executing anything from the file.

    ``.safetensors`` via safetensors; ``.pt/.pth/.bin`` via ``torch.load(weights_only=True)``.
    """
    if path.endswith(".safetensors"):
        from safetensors.numpy import load_file
        return {k: np.asarray(v, dtype=np.float32) for k, v in load_file(path).items()}
    import torch
    sd = torch.load(path, map_location="cpu", weights_only=True)
    return {k: v.detach().float().numpy() for k, v in sd.items()}
