"""Fused EquivariantScalar head (csrc/eq_head.hip): the composite restatement against the
module-by-module blocks on CPU, then the HIP kernel (outputs, per-atom Jacobian, first and second
order gradients) against that composite on the GPU.  Reference: output_modules.py:80-115,
utils.py:456-522."""
import pytest
import torch

from torchmdnet import kernels
from torchmdnet.models.output_modules import EquivariantScalar

DEV = torch.device("cuda", 0)


def _head(H, dtype, seed=0):
    torch.manual_seed(seed)
    head = EquivariantScalar(H, dtype=dtype)
    # non-zero biases so every term is exercised (reset_parameters zeroes them)
    for b in head.output_network:
        for m in (b.update_net[0], b.update_net[2]):
            m.bias.data.normal_(0, 0.3)
    return head


def _inputs(N, H, dtype, device="cpu", seed=1):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(N, H, generator=g, dtype=dtype)
    vec = torch.randn(N, 3, H, generator=g, dtype=dtype)
    vec[2] = 0  # an isolated atom: zero vector features (the reference's masked rows)
    return x.to(device), vec.to(device)


def _blocks(head, x, vec):
    for layer in head.output_network:
        x, vec = layer(x, vec)
    return x + vec.sum() * 0


def test_composite_matches_blocks_cpu():
    head = _head(32, torch.float64)
    assert kernels.eq_head_fusable(head.output_network)
    x, vec = _inputs(7, 32, torch.float64)
    x.requires_grad_(True)
    vec.requires_grad_(True)
    ps = kernels.eq_head_params(head.output_network)
    y_ref = _blocks(head, x, vec)
    y = kernels.eq_head_composite(x, vec, ps)
    assert torch.allclose(y, y_ref, rtol=1e-12, atol=1e-12)
    w = torch.randn_like(y)
    g_ref = torch.autograd.grad((y_ref * w).sum(), [x, vec] + ps)
    g = torch.autograd.grad((y * w).sum(), [x, vec] + ps)
    for a, b in zip(g, g_ref):
        assert torch.isfinite(a).all()
        assert torch.allclose(a, b, rtol=1e-10, atol=1e-12)
    assert torch.all(g[1][2] == 0)  # zero rows get zero gradient, as the reference's mask


def _rel(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.gpu
@pytest.mark.parametrize("nt", ["1", "2"])  # atoms per workgroup (TMDNET_HEAD_NT; 2 from 2k atoms)
@pytest.mark.parametrize("dtype,H,tol", [(torch.float64, 128, 1e-11), (torch.float32, 128, 2e-5),
                                         (torch.float64, 48, 1e-11), (torch.float32, 256, 2e-5)])
def test_hip_head_matches_composite(dtype, H, tol, nt, monkeypatch):
    monkeypatch.setenv("TMDNET_HEAD_NT", nt)
    head = _head(H, dtype).to(DEV)
    ps = kernels.eq_head_params(head.output_network)
    N = 37  # not a multiple of the atom tile
    x, vec = _inputs(N, H, dtype, DEV)
    x.requires_grad_(True)
    vec.requires_grad_(True)
    y = kernels.eq_scalar_head(x, vec, head.output_network)
    y_ref = kernels.eq_head_composite(x, vec, ps)
    assert _rel(y, y_ref) < tol
    gy = torch.randn_like(y)
    # inference-style backward (positions only): the Jacobian path, no weight gradients
    gx, gv = torch.autograd.grad(y, (x, vec), gy, retain_graph=True)
    rx, rv = torch.autograd.grad(y_ref, (x, vec), gy, retain_graph=True)
    assert _rel(gx, rx) < tol and _rel(gv, rv) < tol
    assert torch.all(gv[2] == 0)
    # weight gradients (training's energy term) and second order (force term)
    g1 = torch.autograd.grad(y, [x, vec] + ps, gy, create_graph=True)
    r1 = torch.autograd.grad(y_ref, [x, vec] + ps, gy, create_graph=True)
    for a, b in zip(g1, r1):
        assert _rel(a, b) < tol
    cx, cv = torch.randn_like(x), torch.randn_like(vec)
    l2 = (g1[0] * cx).sum() + (g1[1] * cv).sum()
    m2 = (r1[0] * cx).sum() + (r1[1] * cv).sum()
    g2 = torch.autograd.grad(l2, [x, vec] + ps, allow_unused=True)
    r2 = torch.autograd.grad(m2, [x, vec] + ps, allow_unused=True)
    for a, b in zip(g2, r2):
        if b is None:
            assert a is None or a.abs().max() == 0
            continue
        assert _rel(a, b) < 10 * tol


@pytest.mark.gpu
def test_model_uses_fused_head_and_matches_blocks():
    """create_model's ET + EquivariantScalar routes through the HIP head; energies and forces equal
    the module-by-module head on the same representation (fp64)."""
    from conftest import yaml_args
    from oracle import model_oracle as O
    from torchmdnet.models.model import create_model
    args = yaml_args("equivariant-transformer", embedding_dimension=64, num_layers=2, num_rbf=16, num_heads=4,
                     derivative=True, output_model="Scalar", precision=64)
    torch.manual_seed(3)
    m = create_model(args).to(DEV)
    z, pos, batch = O.qm9_like(6)
    z, pos, batch = z.to(DEV), pos.to(DEV), batch.to(DEV)
    calls = []
    orig = kernels.eq_scalar_head

    def spy(*a):
        calls.append(1)
        return orig(*a)

    kernels.eq_scalar_head = spy
    try:
        y, f = m(z, pos, batch)
    finally:
        kernels.eq_scalar_head = orig
    assert calls
    out = m.output_model
    pr = EquivariantScalar.pre_reduce

    def unfused(self, x, v, z_, pos_, batch_):
        return _blocks(self, x, v)

    EquivariantScalar.pre_reduce = unfused
    try:
        y2, f2 = m(z, pos, batch)
    finally:
        EquivariantScalar.pre_reduce = pr
    assert out is m.output_model
    assert _rel(y, y2) < 1e-11 and _rel(f, f2) < 1e-10


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,H,N,tol", [(torch.float64, 128, 37, 1e-11), (torch.float32, 128, 2100, 5e-5),
                                           (torch.float64, 48, 5, 1e-11)])
def test_head_second_order_hand_matches_composite(dtype, H, N, tol, monkeypatch):
    """tmdnet_eq_head_hvp (forward-over-reverse in one kernel + the weight-term GEMMs) against
    autograd's double differentiation of the composite: the force-loss second order of the head
    for every input (x, vec, the seed g_y) and weight; N = 2100 runs two atoms per workgroup."""
    head = _head(H, dtype).to(DEV)
    ps = kernels.eq_head_params(head.output_network)
    x, vec = _inputs(N, H, dtype, DEV)
    gy = torch.randn(N, 1, dtype=dtype, device=DEV)
    cx, cv = torch.randn_like(x), torch.randn_like(vec)

    def run(mode):
        monkeypatch.setattr(kernels, "HEAD_SECOND_ORDER", mode)
        xs, vs = x.clone().requires_grad_(True), vec.clone().requires_grad_(True)
        g = gy.clone().requires_grad_(True)
        y = kernels.eq_scalar_head(xs, vs, head.output_network)
        gx, gv = torch.autograd.grad(y, (xs, vs), g, create_graph=True)  # the force pass (no weight grads)
        l2 = (gx * cx).sum() + (gv * cv).sum()
        return torch.autograd.grad(l2, [xs, vs, g] + ps, allow_unused=True)

    hand, comp = run("hand"), run("composite")
    for i, (a, b) in enumerate(zip(hand, comp)):
        if b is None or b.abs().max() == 0:
            assert a is None or a.abs().max() == 0, i
            continue
        assert a is not None and torch.isfinite(a).all(), i
        assert _rel(a, b) < tol, (i, _rel(a, b))
    assert torch.all(hand[1][2] == 0)  # the isolated atom's masked rows get nothing of any order


@pytest.mark.gpu
@pytest.mark.parametrize("N", [37, 576, 5003])
def test_mfma_head_matches_valu_kernel_and_fp64(N, monkeypatch):
    """tmdnet_eq_head_x3_f32 (16-atom tiles on the bf16 MFMA, exact three-piece splits; the default fp32
    H = 128 path) against the per-atom VALU kernel (TMDNET_HEAD_X3 off) and the fp64 composite: energies,
    the per-atom Jacobian through the force pass (g_x, g_vec with a random seed), a zero-vector atom
    (the masked norm) and a partial last tile."""
    head = _head(128, torch.float32).to(DEV)
    ps = kernels.eq_head_params(head.output_network)
    x, vec = _inputs(N, 128, torch.float32, DEV)
    gy = torch.randn(N, 1, device=DEV)

    def run(x3):
        monkeypatch.setattr(kernels, "HEAD_X3", x3)
        monkeypatch.setattr(kernels, "HEAD_X3_MIN_ATOMS", 0)
        xx, vv = x.clone().requires_grad_(True), vec.clone().requires_grad_(True)
        y = kernels.eq_scalar_head(xx, vv, head.output_network)
        gx, gv = torch.autograd.grad(y, (xx, vv), gy)
        return y.detach(), gx, gv

    y1, gx1, gv1 = run(True)
    y0, gx0, gv0 = run(False)
    ps64 = [p.detach().double() for p in ps]
    x64, v64 = x.double().requires_grad_(True), vec.double().requires_grad_(True)
    y64 = kernels.eq_head_composite(x64, v64, ps64)
    gx64, gv64 = torch.autograd.grad(y64, (x64, v64), gy.double())
    for a, b, r in ((y1, y0, y64), (gx1, gx0, gx64), (gv1, gv0, gv64)):
        assert _rel(a.double(), r.detach()) < 2e-6
        assert _rel(b.double(), r.detach()) < 2e-6
    assert torch.all(gv1[2] == 0)
