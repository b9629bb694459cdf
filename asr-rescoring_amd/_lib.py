"""ctypes binding of ``librescore.so`` (declared in ``include/rescore.h``).

The library is built in-tree by ``__graft_entry__.build()`` (hipcc, gfx950).  ``torch`` is
imported first so that the HIP runtime ``librescore.so`` links against is the one torch
already loaded (both carry the soname ``libamdhip64.so.7``): device pointers and the
``hipStream_t`` of ``torch.cuda.current_stream()`` are then valid inside the library.
There is no CPU fallback: a missing library or GPU raises.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must load torch's HIP runtime before librescore.so)

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# RS_LIBRESCORE: another in-tree build of the same library (A/B timing of two builds in one GPU
# session); default the library build.py writes.  The override is announced on stderr.
LIB_PATH = os.environ.get("RS_LIBRESCORE") or os.path.join(PKG_DIR, "librescore.so")

RS_HEAD_MLM, RS_HEAD_CLS, RS_HEAD_EMB = 1, 2, 4
RS_FUSE = {"norm": 0, "legacy": 1, "am_norm": 2}
KINDS = ["qkv", "oproj", "ffn1", "ffn2", "decoder", "attn", "other"]


class RsBertCfg(ctypes.Structure):
    _fields_ = [("vocab", ctypes.c_int32), ("hidden", ctypes.c_int32), ("layers", ctypes.c_int32),
                ("heads", ctypes.c_int32), ("intermediate", ctypes.c_int32),
                ("max_pos", ctypes.c_int32), ("type_vocab", ctypes.c_int32),
                ("ln_eps", ctypes.c_float), ("mask_id", ctypes.c_int32),
                ("heads_mask", ctypes.c_int32), ("precision", ctypes.c_int32)]


RS_PREC = {"fp16": 0, "fp16x3": 1}
RS_LOSS = {"MD": 0, "MD_MWER": 1, "MD_MWED": 2}


class RsTrainOpts(ctypes.Structure):
    _fields_ = [("loss", ctypes.c_int32), ("md_loss_weight", ctypes.c_float), ("lr", ctypes.c_float),
                ("beta1", ctypes.c_float), ("beta2", ctypes.c_float), ("eps", ctypes.c_float),
                ("weight_decay", ctypes.c_float), ("update", ctypes.c_int32),
                ("hidden_dropout", ctypes.c_float), ("attn_dropout", ctypes.c_float),
                ("dropout_seed", ctypes.c_uint32)]


class RescoreError(RuntimeError):
    pass


_lib = None
P = ctypes.c_void_p
I32, I64 = ctypes.c_int32, ctypes.c_int64

_SIGS = {
    "rs_version": (ctypes.c_int, []),
    "rs_last_error": (ctypes.c_char_p, []),
    "rs_model_create": (ctypes.c_int, [ctypes.POINTER(RsBertCfg), ctypes.c_int, ctypes.POINTER(P)]),
    "rs_model_set_tensor": (ctypes.c_int, [P, ctypes.c_char_p, P, ctypes.c_int, ctypes.POINTER(I64), ctypes.c_int]),
    "rs_model_finalize": (ctypes.c_int, [P]),
    "rs_model_reserve": (ctypes.c_int, [P, I64]),
    "rs_pll_score": (ctypes.c_int, [P, P, P, I32, P, P, P]),
    "rs_masked_logprob": (ctypes.c_int, [P, P, P, P, P, I32, P, P]),
    "rs_cls_score": (ctypes.c_int, [P, P, P, I32, P, P]),
    "rs_profile_enable": (ctypes.c_int, [P, ctypes.c_int]),
    "rs_profile_read": (ctypes.c_int, [P, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                       ctypes.POINTER(I64), ctypes.POINTER(ctypes.c_double)]),
    "rs_model_set_sync_check": (ctypes.c_int, [P, ctypes.c_int]),
    "rs_check": (ctypes.c_int, [P, P]),
    "rs_model_destroy": (None, [P]),
    "rs_pairwise_edit": (ctypes.c_int, [P, P, P, P, I32, I32, P, P]),
    "rs_mbr_scores": (ctypes.c_int, [P, P, P, P, I32, I32, P, P, P]),
    "rs_mbr_scores_bs": (ctypes.c_int, [P, P, P, I32, I32, I32, P, P, P]),
    "rs_token_embed": (ctypes.c_int, [P, P, P, I32, P, P]),
    "rs_trainer_create": (ctypes.c_int, [ctypes.POINTER(RsBertCfg), ctypes.c_int, ctypes.POINTER(P)]),
    "rs_trainer_set_tensor": (ctypes.c_int, [P, ctypes.c_char_p, P, ctypes.c_int, ctypes.POINTER(I64), ctypes.c_int]),
    "rs_trainer_finalize": (ctypes.c_int, [P]),
    "rs_train_step_cls": (ctypes.c_int, [P, P, P, I32, P, I32, P, P, P, ctypes.POINTER(RsTrainOpts), P, P, P]),
    "rs_train_step_mlm": (ctypes.c_int, [P, P, P, I32, P, P, ctypes.POINTER(RsTrainOpts), P, P]),
    "rs_trainer_get_tensor": (ctypes.c_int, [P, ctypes.c_char_p, P, I64]),
    "rs_trainer_get_grad": (ctypes.c_int, [P, ctypes.c_char_p, P, I64]),
    "rs_trainer_reset_optimizer": (ctypes.c_int, [P]),
    "rs_trainer_dropout_step": (I64, [P]),
    "rs_trainer_set_dropout_step": (ctypes.c_int, [P, I64]),
    "rs_dropout_keep": (ctypes.c_int, [ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_float, I64, P, P]),
    "rs_trainer_destroy": (None, [P]),
    "rs_bertscore_recall": (ctypes.c_int, [P, P, P, P, I32, P, P, P]),
    "rs_align": (ctypes.c_int, [P, P, P, P, I32, P, P, P, P, P, P, P, I32, P]),
    "rs_fuse_rerank": (ctypes.c_int, [P, P, P, P, I32, I32, P, I32, I32, P, P]),
    "rs_corpus_edits": (ctypes.c_int, [P, P, P, I32, I32, P, P]),
    "rs_ref_edit": (ctypes.c_int, [P, P, P, P, P, I32, P, P]),
    "rs_vocab_load": (P, [ctypes.c_char_p]),
    "rs_vocab_size": (ctypes.c_int, [P]),
    "rs_vocab_free": (None, [P]),
    "rs_tokenize_batch": (I64, [P, ctypes.POINTER(ctypes.c_char_p), I32, I32, P, I64, P]),
    "rs_json_write_scores": (ctypes.c_int, [ctypes.c_char_p, I32, ctypes.POINTER(ctypes.c_char_p), P,
                                            ctypes.POINTER(ctypes.c_char_p), P]),
}

# Diagnostic / test entries (not declared in include/rescore.h, not part of the scoring path).
# Typed here so that every caller passes 64-bit pointers: an untyped ctypes call converts a Python
# int to a 32-bit C int, and a truncated device pointer faults the kernel that dereferences it
# (the round-5 "interleaved-W" illegal address: a test called rs_debug_gemm untyped).
CI = ctypes.c_int
_DEBUG_SIGS = {
    "rs_debug_gemm": (CI, [CI, CI, P, P, P, P, CI, CI, CI, P]),
    "rs_debug_attention": (CI, [CI, P, P, P, CI, CI, CI, P, P]),
    "rs_debug_ln": (CI, [CI, CI] + [P] * 9),
    "rs_debug_stamps": (CI, [CI, P]),
    "rs_debug_occupy": (CI, [CI, CI, P, P]),
    "rs_debug_sgemm_cfg": (CI, [CI] * 4 + [P, CI, CI, P, CI, CI, P, CI, CI, P]),
    "rs_debug_sgemm": (CI, [CI] * 3 + [P, CI, CI, P, CI, CI, P, CI, CI, P]),
    "rs_debug_sgemm_pick": (CI, [CI] * 5),
    "rs_debug_gelu": (CI, [P, P, CI, P]),
}
EXPORTED = tuple(_SIGS)          # the shipped library's entries (include/rescore.h)
_SIGS.update(_DEBUG_SIGS)


def load(path: str = LIB_PATH):
    """Load and type the library; raises if it was not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError(f"{path} not found: run `python -c 'import __graft_entry__ as g; g.build()'`")
    if os.environ.get("RS_LIBRESCORE"):
        import sys
        print(f"librescore: RS_LIBRESCORE override {path}", file=sys.stderr)
    lib = ctypes.CDLL(path)
    if not hasattr(lib, "rs_version"):
        raise ImportError(f"{path} is not a librescore build (no rs_version)")
    for name, (res, args) in _SIGS.items():
        if name in _DEBUG_SIGS and not hasattr(lib, name):
            continue                          # RS_DIAG-only entry (rs_debug_stamps) in the shipped build
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int) -> None:
    if rc != 0:
        raise RescoreError(f"librescore error {rc}: {load().rs_last_error().decode()}")


def ptr(t) -> int:
    """Device/host pointer of a tensor or numpy array (None -> NULL)."""
    if t is None:
        return None
    if isinstance(t, torch.Tensor):
        return t.data_ptr()
    return t.ctypes.data


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream
