"""GPU: the ragged self-attention kernels vs a torch fp32 reference (eager_attention_forward,
transformers modeling_bert.py:111-136, scale 64**-0.5, no padding rows), per sequence.

Kernels (k_bert.hip, through the rs_debug_attention diagnostic entry): kind 0 = attn_tr_kernel
(32x32x16 MFMA), kind 6 = attn16_kernel (16x16x32 MFMA, production default).  Lengths cover
the tile edges of both (1, 15/16/17, 31/32/33, 47/48, 63/64/65) and the online-softmax path
(T > 64, several key blocks).  Inputs and P are fp16, accumulation fp32: |err| <= 2e-3 on
O(1) outputs.
"""
import ctypes

import numpy as np
import pytest
import torch

from asr_rescoring_amd import _lib

pytestmark = pytest.mark.gpu

LENGTHS = [1, 2, 3, 15, 16, 17, 31, 32, 33, 34, 47, 48, 49, 63, 64, 65, 96, 100, 128, 130, 200]


def _run(kind, qkv, T, row, H, heads, kx=1):
    lib = _lib.load()
    fn = lib.rs_debug_attention
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 3 + [ctypes.c_int] * 3 + [ctypes.c_void_p] * 2
    dev = qkv.device
    d_len = torch.from_numpy(T).to(dev)
    d_row = torch.from_numpy(row).to(dev)
    ctx = torch.full((qkv.shape[0], kx * H), float("nan"), device=dev, dtype=torch.float16)
    assert fn(kind, qkv.data_ptr(), d_len.data_ptr(), d_row.data_ptr(), len(T), H, heads, ctx.data_ptr(),
              torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    return ctx


@pytest.mark.parametrize("kind", [0, 6])
def test_attention_kernels_vs_torch(kind):
    H, heads = 768, 12
    rng = np.random.default_rng(3)
    T = np.array(LENGTHS * 2, np.int32)
    rng.shuffle(T)
    row = np.concatenate([[0], np.cumsum(T)[:-1]]).astype(np.int32)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(11)
    qkv = (torch.randn(int(T.sum()), 3 * H, device=dev, generator=g) * 0.6).half()
    ctx = _run(kind, qkv, T, row, H, heads)
    worst = 0.0
    for r0, t in zip(row.tolist(), T.tolist()):
        x = qkv[r0:r0 + t].float().view(t, 3, heads, 64)
        q, k, v = x[:, 0].transpose(0, 1), x[:, 1].transpose(0, 1), x[:, 2].transpose(0, 1)
        p = torch.softmax(q @ k.transpose(1, 2) * 0.125, dim=-1)
        ref = (p @ v).transpose(0, 1).reshape(t, H)
        got = ctx[r0:r0 + t].float()
        assert torch.isfinite(got).all(), t
        worst = max(worst, (got - ref).abs().max().item())
    assert worst < 2e-3, worst


def test_attention_kernels_agree():
    """16x16x32 and 32x32x16 kernels on the same C3-like lengths (T 26..44): same result to
    fp16 rounding of P (different key-tile partition of the fp32 sums)."""
    H, heads = 768, 12
    rng = np.random.default_rng(5)
    T = rng.integers(26, 45, size=256).astype(np.int32)
    row = np.concatenate([[0], np.cumsum(T)[:-1]]).astype(np.int32)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(12)
    qkv = (torch.randn(int(T.sum()), 3 * H, device=dev, generator=g) * 0.6).half()
    a = _run(0, qkv, T, row, H, heads).float()
    b = _run(6, qkv, T, row, H, heads).float()
    assert (a - b).abs().max().item() < 2e-3


@pytest.mark.parametrize("kind,tmax", [(9, 64), (10, 48), (11, 64)])
def test_split_precision_attention_vs_torch(kind, tmax):
    """fp16x3 mode: fp32 Q/K/V, ctx written as the [hi | hi/64 | lo*64] operand image.  10 / 11 =
    attn16x3v2_kernel (three fp16 MFMAs per product) with 48 / 64
    staged key rows (swizzled unpadded V image, Vt fragments read per query tile), 9 = fp32
    VALU kernel; all at fp32-level accuracy: |hi + lo - ref| <= 2e-6 on O(1) outputs.
    T <= tmax (the kernel's range)."""
    H, heads = 768, 12
    rng = np.random.default_rng(4)
    T = np.array([t for t in LENGTHS if t <= tmax] * 2, np.int32)
    rng.shuffle(T)
    row = np.concatenate([[0], np.cumsum(T)[:-1]]).astype(np.int32)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(13)
    qkv = torch.randn(int(T.sum()), 3 * H, device=dev, generator=g) * 0.6
    ctx = _run(kind, qkv, T, row, H, heads, kx=3).float()
    got_all = ctx[:, :H] + ctx[:, 2 * H:] / 64
    assert torch.equal((ctx[:, :H] / 64).half().float(), ctx[:, H:2 * H])     # mid = fp16(hi / 64)
    worst = 0.0
    for r0, t in zip(row.tolist(), T.tolist()):
        x = qkv[r0:r0 + t].double().view(t, 3, heads, 64)
        q, k, v = x[:, 0].transpose(0, 1), x[:, 1].transpose(0, 1), x[:, 2].transpose(0, 1)
        p = torch.softmax(q @ k.transpose(1, 2) * 0.125, dim=-1)
        ref = (p @ v).transpose(0, 1).reshape(t, H)
        worst = max(worst, (got_all[r0:r0 + t].double() - ref).abs().max().item())
    assert worst < 2e-6, worst
