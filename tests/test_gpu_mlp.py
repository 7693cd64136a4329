"""GPU checks of kernels.mlp_act (tmdnet_gemm_ex_f32: Linear + SiLU stacks with the activation, the
pre-activation store, the row scale and the backward chain's silu' in the GEMM epilogues) against the
fp64 composite of the reference's Linear -> act loops (tensornet.py:233, 320-321, 381-385): values,
first-order gradients of every input, and the second order the force-matching loss takes."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return float((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30))


def _inputs(rows, dims, scaled, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(rows, dims[0], generator=g)
    ws = [torch.randn(dims[i + 1], dims[i], generator=g) / dims[i] ** 0.5 for i in range(len(dims) - 1)]
    bs = [torch.randn(dims[i + 1], generator=g) * 0.1 for i in range(len(dims) - 1)]
    sc = torch.rand(rows, generator=g) if scaled else None
    return x, ws, bs, sc


@pytest.mark.parametrize("rows,dims,scaled", [(3360, (32, 128, 256, 384), True), (168, (128, 128, 128), False),
                                              (168, (384, 128), False), (37, (16, 48, 32), True)])
def test_mlp_act_matches_composite(rows, dims, scaled):
    from torchmdnet import kernels
    x, ws, bs, sc = _inputs(rows, dims, scaled)
    calls = []
    orig = kernels.gemm_ex_launch

    def counting(p):
        calls.append(len(p))
        return orig(p)
    kernels.gemm_ex_launch = counting
    try:
        def run(dtype, fused):
            t = [v.to(DEV, dtype).requires_grad_(True) for v in [x] + ws + bs]
            s = sc.to(DEV, dtype).requires_grad_(True) if sc is not None else None
            L = len(ws)
            if fused:
                y = kernels.mlp_act(t[0], t[1:1 + L], t[1 + L:], torch.nn.SiLU(), s)
            else:
                y = kernels._mlp_composite(t[0], s, *t[1:])
            gy = torch.randn(y.shape, generator=torch.Generator().manual_seed(3)).to(DEV, dtype)
            prim = t + ([s] if s is not None else [])
            g1 = torch.autograd.grad(y, prim, gy, create_graph=True)
            # second order: a scalar of the first-order gradients differentiated again (force-loss shape)
            tot = sum((gi * gi).sum() for gi in g1)
            g2 = torch.autograd.grad(tot, prim)
            return y.detach(), [v.detach() for v in g1], [v.detach() for v in g2]
        y, g1, g2 = run(torch.float32, True)
        assert calls, "the fused GEMM path did not run"
        y64, g164, g264 = run(torch.float64, False)
    finally:
        kernels.gemm_ex_launch = orig
    assert _rel(y, y64) < 1e-5
    for a, b in zip(g1, g164):
        assert _rel(a, b) < 1e-5
    for a, b in zip(g2, g264):
        assert _rel(a, b) < 1e-4


def test_mlp_act_falls_back_outside_envelope():
    """Rows above the GEMM envelope, K not a multiple of 16, fp64: Linear + fused_act per layer."""
    from torchmdnet import kernels
    x, ws, bs, sc = _inputs(50, (20, 32, 16), True)
    xs = [v.to(DEV) for v in [x] + ws + bs]
    y = kernels.mlp_act(xs[0], xs[1:3], xs[3:], torch.nn.SiLU(), sc.to(DEV))
    ref = kernels._mlp_composite(xs[0].double(), sc.to(DEV).double(), *[v.double() for v in xs[1:]])
    assert _rel(y, ref) < 1e-5
