"""Diagnostic: split-precision attention (attn16x3v2, kind 11) vs fp32 VALU (kind 9), fp16 kernel (kind 6) and fp64 torch."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import __graft_entry__  # noqa: E402

__graft_entry__._import_pkg()
from test_gpu_attention import _run  # noqa: E402

H, heads = 768, 12
T = np.array([34, 17, 64, 5], np.int32)
row = np.concatenate([[0], np.cumsum(T)[:-1]]).astype(np.int32)
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(13)
for scale in (0.6, 60.0):
    qkv = torch.randn(int(T.sum()), 3 * H, device=dev, generator=g) * scale
    if scale > 1:
        qkv[:, :2 * H] *= 0.6 / scale          # keep scores O(1); only V large
    x = qkv.double().view(-1, 3, heads, 64)
    refs = []
    for r0, t in zip(row.tolist(), T.tolist()):
        xx = x[r0:r0 + t]
        q, k, v = xx[:, 0].transpose(0, 1), xx[:, 1].transpose(0, 1), xx[:, 2].transpose(0, 1)
        p = torch.softmax(q @ k.transpose(1, 2) * 0.125, dim=-1)
        refs.append((p @ v).transpose(0, 1).reshape(t, H))
    ref = torch.cat(refs)
    c8 = _run(11, qkv, T, row, H, heads, kx=3).double()
    c9 = _run(9, qkv, T, row, H, heads, kx=3).double()
    c6 = _run(6, qkv.half(), T, row, H, heads).double()
    o8 = c8[:, :H] + c8[:, 2 * H:] / 64
    o9 = c9[:, :H] + c9[:, 2 * H:] / 64
    print(f"scale {scale}: |k8-ref| {(o8 - ref).abs().max().item():.3e}  |k9-ref| {(o9 - ref).abs().max().item():.3e}  "
          f"|k6-ref| {(c6 - ref).abs().max().item():.3e}  |k8hi-k6| {(c8[:, :H] - c6).abs().max().item():.3e}  "
          f"|k8lo| max {c8[:, 2 * H:].abs().max().item():.3e}", flush=True)
