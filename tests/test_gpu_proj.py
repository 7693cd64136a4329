"""GPU checks of ``tmdnet_proj_f32`` (the dk/dv projection of the pair rows on the bf16 MFMA with an
exact three-piece operand split, csrc/gemm.hip ``tmd::proj``), reference torchmd_et.py:282-291.

The kernel claims fp32 GEMM accuracy, so the bar is relative to the library fp32 GEMM on the same
inputs: its error against an fp64 product must not exceed the library's by more than 2x (plus a few
fp32 ulps of the output scale).  Shapes: the model's (pair rows x 8 stacked layers, per-layer, the
adjoint without bias), ragged M (tails of the 16-row blocks and 128-row tiles), strided operands /
output (the stacked pkv_all slices), K = 32 and 64; outside the envelope the wrapper must fall back to
the library GEMM (same result as torch).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _check(A, W, b, out=None):
    from torchmdnet import kernels
    got = kernels.proj(A, W, b, out=out)
    ref = A.double() @ W.double().t()
    if b is not None:
        ref = ref + b.double()
    lib = (torch.addmm(b, A, W.t()) if b is not None else A @ W.t()).double()
    e_lib = float((lib - ref).abs().max())
    e_got = float((got.double() - ref).abs().max())
    scale = float(ref.abs().max())
    assert e_got <= 2 * e_lib + 4 * 2.0 ** -24 * scale, (e_got, e_lib, scale)
    return got


@pytest.mark.parametrize("M", [1, 17, 200, 6613])
@pytest.mark.parametrize("N", [16, 512, 4096])
@pytest.mark.parametrize("K", [32, 64])
@pytest.mark.parametrize("bias", [True, False])
def test_proj_matches_fp64_like_library(M, N, K, bias):
    torch.manual_seed(M + N + K)
    A = torch.rand(M, K, device=DEV)  # RBF rows: [0, 1]
    W = torch.randn(N, K, device=DEV) / K ** 0.5
    b = torch.randn(N, device=DEV) if bias else None
    _check(A, W, b)


@pytest.mark.parametrize("K", [32, 64])
def test_proj_large_tile_config(K):
    """M >= 65536 selects the large tiles (256 rows; 128 columns at K = 64, 64 at K = 32 -- the grid
    must follow the tile actually launched: every column written), ragged M."""
    torch.manual_seed(2)
    A = torch.rand(70001, K, device=DEV)
    W = torch.randn(512, K, device=DEV) / K ** 0.5
    out = torch.full((70001, 512), float("nan"), device=DEV)
    got = _check(A, W, torch.randn(512, device=DEV), out=out)
    assert bool(torch.isfinite(got).all())


def test_proj_strided_operands_and_output():
    torch.manual_seed(1)
    M, N, K = 3001, 1024, 64
    A = torch.randn(M, K + 12, device=DEV)[:, 4:4 + K]  # lda = 76, 16-byte aligned rows
    W = torch.randn(N, K + 4, device=DEV)[:, :K]
    b = torch.randn(2 * N, device=DEV)[N:]
    out = torch.full((M, N + 32), 7.0, device=DEV)
    got = _check(A, W, b, out=out[:, 16:16 + N])
    assert got.data_ptr() == out[:, 16:].data_ptr()
    assert torch.all(out[:, :16] == 7.0) and torch.all(out[:, 16 + N:] == 7.0)


def test_proj_row_slice_of_a_shared_split():
    """A layer's rows of the stacked weight through the stacked split (et_stack.Meta.dkv_proj)."""
    from torchmdnet import kernels
    torch.manual_seed(4)
    M, D, L, K = 999, 512, 3, 64
    A, W, b = torch.rand(M, K, device=DEV), torch.randn(L * D, K, device=DEV) / 8, torch.randn(L * D, device=DEV)
    wp = kernels.proj_split(W)
    assert wp is not None and wp.shape == (3, L * D, K)
    # the split is exact: the pieces sum back to W
    parts = [(wp[i].to(torch.int32) & 0xFFFF).to(torch.int32) << 16 for i in range(3)]
    back = sum(p.view(torch.float32).double() for p in parts)
    assert torch.equal(back, W.double())
    for l in range(L):
        got = kernels.proj(A, W[l * D:(l + 1) * D], b[l * D:(l + 1) * D], wp=wp, row0=l * D)
        ref = kernels.proj(A, W[l * D:(l + 1) * D], b[l * D:(l + 1) * D])
        assert torch.equal(got, ref)
        _check(A, W[l * D:(l + 1) * D], b[l * D:(l + 1) * D])


def test_proj_extreme_magnitudes():
    """The split is exact for every normal fp32 value: mixed magnitudes keep fp32 accuracy."""
    torch.manual_seed(2)
    M, N, K = 333, 256, 64
    A = torch.randn(M, K, device=DEV) * torch.exp2(torch.randint(-20, 20, (M, K), device=DEV).float())
    W = torch.randn(N, K, device=DEV) * torch.exp2(torch.randint(-10, 10, (N, K), device=DEV).float())
    _check(A, W, None)


def test_proj_outside_envelope_falls_back():
    from torchmdnet import kernels
    torch.manual_seed(3)
    A, W = torch.randn(100, 48, device=DEV), torch.randn(80, 48, device=DEV)  # K = 48
    assert torch.equal(kernels.proj(A, W), A @ W.t())
    A, W = torch.randn(100, 64, device=DEV), torch.randn(24, 64, device=DEV)  # N % 16 != 0
    assert torch.equal(kernels.proj(A, W), A @ W.t())
    Ad, Wd = A.double(), torch.randn(32, 64, device=DEV, dtype=torch.float64)
    assert torch.equal(kernels.proj(Ad, Wd), Ad @ Wd.t())


# ----------------------------------------------------------------------------- large-row node-mix GEMM
@pytest.mark.parametrize("M", [16385, 50001])
@pytest.mark.parametrize("N,K,tb", [(640, 128, True), (384, 128, True), (64, 128, True), (128, 640, False),
                                    (128, 384, False), (64, 128, False), (144, 96, True)])
@pytest.mark.parametrize("bias,beta", [(True, False), (False, True)])
def test_gemm_x3_large_rows_match_fp64_like_library(M, N, K, tb, bias, beta):
    """tmdnet_gemm_x3_f32 (the node feature mixes above GEMM_MAX_ROWS: the forward Linears with a [N][K]
    weight and the input gradients g W with an untransposed [K][N] right operand, K chunked by 128 / 64,
    ragged M) against fp64: no worse than 2x the library fp32 GEMM's error plus a few output ulps;
    beta accumulates into C."""
    from torchmdnet import kernels
    torch.manual_seed(M + N + K)
    A = torch.randn(M, K, device=DEV)
    B = torch.randn(N, K, device=DEV) / K ** 0.5 if tb else torch.randn(K, N, device=DEV) / K ** 0.5
    b = torch.randn(N, device=DEV) if bias else None
    C0 = torch.randn(M, N, device=DEV)
    C = C0.clone()
    assert kernels.gemm_x3(A, B, tb, b, C, beta)
    Bop = B.t() if tb else B
    ref = A.double() @ Bop.double()
    lib = A @ Bop
    if b is not None:
        ref = ref + b.double()
        lib = lib + b
    if beta:
        ref = ref + C0.double()
        lib = lib + C0
    e_lib = float((lib.double() - ref).abs().max())
    e_got = float((C.double() - ref).abs().max())
    scale = float(ref.abs().max())
    assert e_got <= 2 * e_lib + 4 * 2.0 ** -24 * scale, (e_got, e_lib, scale)


def test_gemm_group_large_rows_takes_the_x3_kernel(monkeypatch):
    """gemm_group above GEMM_MAX_ROWS: every fp32 problem on tmdnet_gemm_x3_f32 (no library GEMM)."""
    from torchmdnet import kernels
    seen = []
    orig = kernels.gemm_x3
    monkeypatch.setattr(kernels, "gemm_x3", lambda *a: seen.append(1) or orig(*a))
    monkeypatch.setattr(torch, "mm", lambda *a, **k: (_ for _ in ()).throw(AssertionError("library GEMM")))
    monkeypatch.setattr(torch, "addmm", lambda *a, **k: (_ for _ in ()).throw(AssertionError("library GEMM")))
    M = kernels.GEMM_MAX_ROWS + 100
    A = torch.randn(M, 128, device=DEV)
    W1, W2 = torch.randn(640, 128, device=DEV), torch.randn(384, 128, device=DEV)
    C1, C2 = torch.empty(M, 640, device=DEV), torch.empty(M, 384, device=DEV)
    kernels.gemm_group([(A, W1, True, None, C1, False), (A, W2, True, None, C2, False)])
    assert len(seen) == 2
