"""GPU: the fp16 MFMA GEMM kernels (k_gemm.hip) through the rs_debug_gemm diagnostic entry.

* every production variant vs a torch fp32 reference of the same op (C = A.W^T + bias, GELU);
* the persistent kernel's wave schedule (younger half at s_setprio 1 and one MFMA substep behind,
  wave-private epilogue slabs without the epilogue barrier) is BITWISE equal to the
  barrier-synchronised baseline — the same MFMA order per accumulator — on fresh random inputs
  (the race screen of tools/diag/gemm_race_screen.py, reduced).
"""
import ctypes

import pytest
import torch

from asr_rescoring_amd import _lib

pytestmark = pytest.mark.gpu

# rs_debug_gemm cfg: 9 / 11 persistent bias / GELU, VAR 0; 21 bias, 18 GELU = production schedule;
# 0 with dbg 8384 = pipelined plain kernel (16x16x32, non-temporal stores)
SHAPES = [("qkv", 2304, 768, False), ("oproj", 768, 768, False), ("ffn1", 3072, 768, True),
          ("ffn2", 768, 3072, False)]


@pytest.fixture(scope="module")
def gemm():
    lib = _lib.load()
    fn = lib.rs_debug_gemm
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_int] * 3 + [ctypes.c_void_p]
    st = torch.cuda.current_stream().cuda_stream

    def run(cfg, dbg, A, W, b, out):
        M, K = A.shape
        N = W.shape[0]
        assert fn(cfg, dbg, A.data_ptr(), W.data_ptr(), b.data_ptr(), out.data_ptr(), M, N, K, st) == 0
        torch.cuda.synchronize()
        return out
    return run


def _operands(M, N, K, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    A = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).half()
    W = (torch.rand(N, K, device="cuda", generator=g) * 2 - 1).half()
    b = torch.rand(N, device="cuda", generator=g)
    return A, W, b


@pytest.mark.parametrize("name,N,K,gelu", SHAPES)
def test_gemm_variants_vs_torch(gemm, name, N, K, gelu):
    M = 4096
    A, W, b = _operands(M, N, K, 3)
    ref = A.float() @ W.float().t() + b
    if gelu:
        ref = torch.nn.functional.gelu(ref)
    cfgs = [(11, 0), (18, 0)] if gelu else [(9, 0), (21, 0), (0, 8384)]
    for cfg, dbg in cfgs:
        out = gemm(cfg, dbg, A, W, b, torch.full((M, N), float("nan"), device="cuda", dtype=torch.float16))
        # fp16 output rounding (|C| up to ~sqrt(K)) + fp32 accumulation-order differences
        err = (out.float() - ref).abs() / ref.abs().clamp_min(1.0)
        assert err.max().item() < 2e-3, (name, cfg, dbg, err.max().item())


@pytest.mark.parametrize("name,N,K,gelu", SHAPES)
def test_persistent_schedule_bitwise(gemm, name, N, K, gelu):
    prod, base = (18, 11) if gelu else (21, 9)
    M = 256 * 131                 # 131 row panels: a partial last wave of tiles
    for rep in range(3):
        A, W, b = _operands(M, N, K, 100 + rep)
        o1 = gemm(prod, 0, A, W, b, torch.full((M, N), float("nan"), device="cuda", dtype=torch.float16))
        o2 = gemm(base, 0, A, W, b, torch.full((M, N), float("nan"), device="cuda", dtype=torch.float16))
        assert torch.equal(o1.view(torch.int16), o2.view(torch.int16)), (name, rep)
