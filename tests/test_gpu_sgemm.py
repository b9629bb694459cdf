"""GPU: the trainer's fp32 GEMM (k_sgemm.hip, f32-input MFMA) through rs_debug_sgemm.

The three operand forms a Linear's forward / backward needs (RescoreBert/main.py:104-150 and
MLM_PLL/main.py:89-97 train transformers' BertModel in fp32):
  forward  Y  = X · Wᵀ,  dgrad  dX = dY · W,  wgrad  dW = dYᵀ · X
against a float64 torch product of the same fp32 operands, on ragged shapes (token counts that
are not tile multiples), with and without accumulation into C, on both sides of the split-K
switch; plus bitwise reproducibility (no atomics) and untouched memory outside C's rows.
"""
import ctypes

import pytest
import torch

from asr_rescoring_amd import _lib

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sgemm():
    lib = _lib.load()
    fn = lib.rs_debug_sgemm_cfg
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    st = torch.cuda.current_stream().cuda_stream

    def run(form, dY_or_X, W_or_X, out, accum, cfg=-1):
        """form nt: out[M,N] = A[M,K] . B[N,K]^T; nn: out[M,K] = A[M,N] . B[N,K];
        tn: out[N,K] = A[M,N]^T . B[M,K].  cfg: tile configuration (-1: the shape's pick)."""
        A, B = dY_or_X, W_or_X
        if form == "nt":
            M, K = A.shape
            N = B.shape[0]
            r = fn(cfg, M, N, K, A.data_ptr(), K, 1, B.data_ptr(), K, 1, out.data_ptr(), out.stride(0), accum, st)
        elif form == "nn":
            M, N = A.shape
            K = B.shape[1]
            r = fn(cfg, M, K, N, A.data_ptr(), N, 1, B.data_ptr(), K, 0, out.data_ptr(), out.stride(0), accum, st)
        else:
            M, N = A.shape
            K = B.shape[1]
            r = fn(cfg, N, K, M, A.data_ptr(), N, 0, B.data_ptr(), K, 0, out.data_ptr(), out.stride(0), accum, st)
        assert r == 0
        torch.cuda.synchronize()
        return out
    return run


def _ref(form, A, B):
    A64, B64 = A.double(), B.double()
    if form == "nt":
        return A64 @ B64.t()
    if form == "nn":
        return A64 @ B64
    return A64.t() @ B64


def _abs_bound(form, A, B):
    """fp32 accumulation bound per element: ~K ulp of sum |a||b| (k-ordered fmaf chain + split sum)"""
    Aa, Ba = A.double().abs(), B.double().abs()
    s = _ref(form, Aa, Ba)
    K = A.shape[1] if form in ("nt", "nn") else A.shape[0]
    return s * (2.0 ** -24) * (4 + K ** 0.5 * 2)


# (form, rows M, N, K): forward / dgrad / wgrad of the BERT-base Linears at a ragged token count,
# the tied MLM decoder, and small tile counts (split-K) vs many tiles (one pass)
CASES = [("nt", 1037, 2304, 768), ("nt", 1037, 768, 3072), ("nt", 301, 21128, 768), ("nt", 77, 768, 768),
         ("nn", 1037, 768, 2304), ("nn", 1037, 3072, 768), ("nn", 130, 768, 21128),
         ("tn", 1037, 2304, 768), ("tn", 1037, 768, 3072), ("tn", 4999, 768, 768), ("tn", 33, 3072, 768)]


@pytest.mark.parametrize("form,M,N,K", CASES)
@pytest.mark.parametrize("accum", [0, 1])
@pytest.mark.parametrize("cfg", [0, "streamk", 9, 11, 12, 17, 18])
def test_sgemm_forms_vs_float64(sgemm, form, M, N, K, accum, cfg, monkeypatch):
    """Every live tile configuration (k_sgemm.hip kSgCfg) on every form and edge, and the opt-in
    stream-K form of cfg 0 (RS_SGEMM_SK=1: partial tiles handed between workgroups)."""
    if cfg == "streamk":
        monkeypatch.setenv("RS_SGEMM_SK", "1")
        cfg = 0
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N + K)
    if form == "nt":
        A = torch.randn(M, K, device="cuda", generator=g)
        B = torch.randn(N, K, device="cuda", generator=g) * 0.05
        shape = (M, N)
    elif form == "nn":       # A = dY [M, N'], B = W [N', K]: here N is the Linear's out, K its in
        A = torch.randn(M, N, device="cuda", generator=g) * 1e-3
        B = torch.randn(N, K, device="cuda", generator=g) * 0.05
        shape = (M, K)
    else:                    # A = dY [M, N], B = X [M, K]
        A = torch.randn(M, N, device="cuda", generator=g) * 1e-3
        B = torch.randn(M, K, device="cuda", generator=g)
        shape = (N, K)
    C0 = torch.randn(*shape, device="cuda", generator=g) if accum else \
        torch.full(shape, float("nan"), device="cuda")
    ref = _ref(form, A, B) + (C0.double() if accum else 0.0)
    out = sgemm(form, A, B, C0.clone(), accum, cfg)
    err = (out.double() - ref).abs()
    bound = _abs_bound(form, A, B) + (C0.double().abs() * 2.0 ** -23 if accum else 0.0)
    assert torch.isfinite(out).all()
    assert (err <= bound).all(), (form, M, N, K, float((err / bound).max()))
    # same inputs, same bits (ordered split-K sum, no atomics)
    again = sgemm(form, A, B, C0.clone(), accum, cfg)
    assert torch.equal(out, again)


def test_sgemm_retired_configurations_fail():
    """Retired tile configurations (measured, never picked, instantiations removed) keep their
    index and fail the call instead of running something else."""
    lib = _lib.load()
    fn = lib.rs_debug_sgemm_cfg
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    A = torch.randn(64, 64, device="cuda")
    B = torch.randn(64, 64, device="cuda")
    C = torch.zeros(64, 64, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    for cfg in (1, 3, 4, 10, 13, 15, 16, 19, 20):
        assert fn(cfg, 64, 64, 64, A.data_ptr(), 64, 1, B.data_ptr(), 64, 1, C.data_ptr(), 64, 0, st) != 0, cfg
    torch.cuda.synchronize()
    assert torch.all(C == 0)


def test_sgemm_leaves_padding_columns_alone(sgemm):
    """C with a row stride wider than N: columns past N are never written."""
    M, N, K = 200, 132, 96
    A = torch.randn(M, K, device="cuda")
    B = torch.randn(N, K, device="cuda")
    Cw = torch.full((M, N + 60), 7.0, device="cuda")
    sgemm("nt", A, B, Cw[:, :N], 0)
    assert torch.all(Cw[:, N:] == 7.0)
    torch.testing.assert_close(Cw[:, :N], (A.double() @ B.double().t()).float(), rtol=1e-5, atol=1e-4)


def test_sgemm_matches_torch_fp32_linear_backward(sgemm):
    """The three forms together reproduce torch.nn.Linear's fp32 autograd (the trainer's use)."""
    M, I, O = 517, 768, 3072
    X = torch.randn(M, I, device="cuda", requires_grad=True)
    lin = torch.nn.Linear(I, O, bias=False).cuda()
    Y = lin(X)
    dY = torch.randn_like(Y) * 1e-2
    Y.backward(dY)
    with torch.no_grad():
        y = sgemm("nt", X.detach(), lin.weight.detach(), torch.empty(M, O, device="cuda"), 0)
        dx = sgemm("nn", dY, lin.weight.detach(), torch.empty(M, I, device="cuda"), 0)
        dw = sgemm("tn", dY, X.detach(), torch.empty(O, I, device="cuda"), 0)
    for mine, ref in ((y, Y.detach()), (dx, X.grad), (dw, lin.weight.grad)):
        rel = float((mine - ref).norm() / ref.norm())
        assert rel < 1e-5, rel
