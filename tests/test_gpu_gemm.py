"""GPU: the fp16 MFMA GEMM kernels (k_gemm.hip) through the rs_debug_gemm diagnostic entry.

* every production variant vs a torch fp32 reference of the same op (C = A.W^T + bias, GELU);
* the persistent kernel's wave schedule (younger half at s_setprio 1 and one MFMA substep behind,
  wave-private epilogue slabs without the epilogue barrier) is BITWISE equal to the
  barrier-synchronised baseline — the same MFMA order per accumulator — on fresh random inputs
  (a reduced race screen).
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


def _split2(x):
    hi = x.half()
    return torch.cat([hi, ((x - hi.float()) * 64.0).half()], dim=1).contiguous()


@pytest.mark.parametrize("dbg,M", [(0, 1024), (0, 40960)])
@pytest.mark.parametrize("name,N,K,gelu", SHAPES)
def test_x3s_vs_torch_fp32(gemm, name, N, K, gelu, dbg, M):
    """Split-operand fp16x3 GEMM (cfg 31/32 of rs_debug_gemm, dbg 0 = gemm_x3s_kernel): fp32 output and the two-part GELU image vs an fp32 torch matmul, at
    fp32-level accuracy (3 fp16 products; measured ~2e-6 of max |C|).  M = 40960 gives every
    persistent workgroup several tiles (tile transitions, the last tile of each workgroup)."""
    g = torch.Generator(device="cuda").manual_seed(11)
    A = torch.randn(M, K, device="cuda", generator=g)
    W = torch.randn(N, K, device="cuda", generator=g) * 0.05
    b = torch.randn(N, device="cuda", generator=g) * 0.1
    A2, W2 = _split2(A), _split2(W)
    ref = A @ W.t() + b
    lib = _lib.load()          # direct call: the logical K (the fixture passes A's width)
    st = torch.cuda.current_stream().cuda_stream
    for cfg, o in ((32, torch.empty(M, N, device="cuda")), (31, torch.empty(M, 2 * N, device="cuda", dtype=torch.float16))):
        assert lib.rs_debug_gemm(cfg, dbg, A2.data_ptr(), W2.data_ptr(), b.data_ptr(), o.data_ptr(), M, N, K, st) == 0
        torch.cuda.synchronize()
        if cfg == 32:
            err = (o - ref).abs().max() / ref.abs().max()
        else:
            gl = torch.nn.functional.gelu(ref)
            err = (o[:, :N].float() + o[:, N:].float() / 64.0 - gl).abs().max() / gl.abs().max()
        assert err < 1e-5, (cfg, float(err))
