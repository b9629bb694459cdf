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

    def run(cfg, dbg, A, W, b, out, K=None):
        M = A.shape[0]
        K = A.shape[1] if K is None else K          # split-operand cfg 31/32: the logical K
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
    """The split-operand GEMM's two-part image of fp32 x [R, K] (common.h kx == 2): hi and
    lo = (x - hi) * 64 interleaved per 32-column K-step, [hi 0..31 | lo 0..31 | hi 32..63 | ...]."""
    hi = x.half()
    lo = ((x - hi.float()) * 64.0).half()
    R, K = x.shape
    return torch.stack([hi.view(R, K // 32, 32), lo.view(R, K // 32, 32)], dim=2).reshape(R, 2 * K).contiguous()


def _unsplit2(img):
    """hi + lo / 64 of an interleaved two-part image [R, 2N] -> fp32 [R, N]."""
    R, N2 = img.shape
    v = img.float().view(R, N2 // 64, 2, 32)
    return (v[:, :, 0] + v[:, :, 1] / 64.0).reshape(R, N2 // 2)


def test_split2_layout():
    x = torch.arange(2 * 64, dtype=torch.float32).view(2, 64) + 0.25
    img = _split2(x)
    assert torch.equal(img[0, :32].float(), x[0, :32].half().float())          # hi of columns 0..31
    assert torch.equal(img[0, 64:96].float(), x[0, 32:].half().float())        # hi of columns 32..63
    assert torch.allclose(_unsplit2(img), x)


@pytest.mark.parametrize("dbg,M", [(0, 1024), (0, 40960)])
@pytest.mark.parametrize("name,N,K,gelu", SHAPES)
def test_x3s_vs_torch_fp32(gemm, name, N, K, gelu, dbg, M):
    """Split-operand fp16x3 GEMM (cfg 31/32 of rs_debug_gemm, dbg 0 = gemm_x3s_kernel) on the
    interleaved two-part images: fp32 output and the GELU image vs an fp32 torch matmul, at
    fp32-level accuracy (3 fp16 products; measured ~2e-6 of max |C|).  M = 40960 gives every
    persistent workgroup several tiles (tile transitions, the last tile of each workgroup);
    M = 1024 one tile per workgroup (the first tile is the last)."""
    g = torch.Generator(device="cuda").manual_seed(11)
    A = torch.randn(M, K, device="cuda", generator=g)
    W = torch.randn(N, K, device="cuda", generator=g) * 0.05
    b = torch.randn(N, device="cuda", generator=g) * 0.1
    A2, W2 = _split2(A), _split2(W)
    ref = A @ W.t() + b
    for cfg, o in ((32, torch.empty(M, N, device="cuda")), (31, torch.empty(M, 2 * N, device="cuda", dtype=torch.float16))):
        gemm(cfg, dbg, A2, W2, b, o, K=K)
        if cfg == 32:
            err = (o - ref).abs().max() / ref.abs().max()
        else:
            gl = torch.nn.functional.gelu(ref)
            err = (_unsplit2(o) - gl).abs().max() / gl.abs().max()
        assert err < 1e-5, (cfg, float(err))


@pytest.mark.parametrize("M", [1024, 40960, 262144])
@pytest.mark.parametrize("name,N,K,gelu", SHAPES[:3])
def test_x3s_deterministic_at_tile_counts(gemm, name, N, K, gelu, M):
    """Interleaved split-operand GEMM: bitwise run-to-run determinism at M = 1024 (36 / 12 workgroups
    of one tile each: the first tile is the last — the round-5 fault case, whose cause was an untyped
    ctypes call truncating the pointers, not the kernel), 40960 and 262144 (many tiles per workgroup),
    and fp32-level agreement with torch on the first rows."""
    g = torch.Generator(device="cuda").manual_seed(17)
    A = torch.randn(M, K, device="cuda", generator=g)
    W = torch.randn(N, K, device="cuda", generator=g) * 0.05
    b = torch.randn(N, device="cuda", generator=g) * 0.1
    A2, W2 = _split2(A), _split2(W)
    outs = []
    for _ in range(2):
        o = torch.full((M, N), float("nan"), device="cuda")
        gemm(32, 0, A2, W2, b, o, K=K)
        outs.append(o)
    assert torch.equal(outs[0].view(torch.int32), outs[1].view(torch.int32))
    ref = A[:4096] @ W.t() + b
    assert (outs[0][:4096] - ref).abs().max() / ref.abs().max() < 1e-5


def test_gelu_vs_torch_fp32():
    """The epilogues' GELU (gemm_dev.h gelu2: relu(x) - a erfc(a/sqrt2)/2 with erfc/2 = 2^P(a),
    a = min(|x|, 5.7 sqrt2)) evaluated elementwise in fp32 against the exact erf GELU (torch, fp64):
    |error| <= 3e-7 over the whole input range — dense on [-12, 12], sparse out to +-1e30, and the
    special points (0, +-AMAX, subnormals); non-finite inputs stay non-finite."""
    lib = _lib.load()
    dense = torch.linspace(-12, 12, 4_000_001, dtype=torch.float32)
    wide = torch.logspace(-30, 30, 200_001, dtype=torch.float32)
    special = torch.tensor([0.0, -0.0, 8.06101731, -8.06101731, 1e-40, -1e-40, 5.7 * 2 ** 0.5, 3.0e38, -3.0e38],
                           dtype=torch.float32)
    x = torch.cat([dense, wide, -wide, special]).cuda()
    y = torch.empty_like(x)
    assert lib.rs_debug_gelu(x.data_ptr(), y.data_ptr(), x.numel(), torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    ref = torch.nn.functional.gelu(x.double())
    err = (y.double() - ref).abs()
    assert err.max().item() <= 3e-7, (err.max().item(), x[err.argmax()].item())
    # a non-finite pre-activation (an operand image that overflowed fp16) must stay non-finite,
    # so that the scoring call's range guard reports it instead of scoring a silently clamped value
    bad = torch.tensor([float("inf"), float("-inf"), float("nan")], device="cuda")
    yb = torch.empty_like(bad)
    assert lib.rs_debug_gelu(bad.data_ptr(), yb.data_ptr(), 3, torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    assert not torch.isfinite(yb).any(), yb
