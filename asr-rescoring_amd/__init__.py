"""MI355X-native N-best LM rescorer (MLM_PLL / RescoreBert / RMBR-CER + fusion).

Host side in Python over a C-ABI library ``librescore.so`` (HIP kernels for gfx950).
The library is loaded lazily by the scoring classes; importing the package itself does
not touch the GPU, so the pure host modules (``data``, ``weights``, ``config``) work on CPU.
"""
from . import data, weights  # noqa: F401

__all__ = ["data", "weights", "PLLScorer", "RescoreBertHIP", "fuse_rerank", "mbr_decode"]


def __getattr__(name):
    if name in ("PLLScorer", "RescoreBertHIP", "BertEngine"):
        from . import scorer
        return getattr(scorer, name)
    if name in ("fuse_rerank", "find_best_weight", "mbr_decode", "find_best_length",
                "pairwise_edit", "corpus_edits"):
        from . import rerank
        return getattr(rerank, name)
    raise AttributeError(name)
