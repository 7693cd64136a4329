"""Hand kernels of the TensorNet / Scalar-head tail (VERDICT r3 "next" #7) against their composites:
LayerNorm (tmdnet_layernorm_*: reference nn.LayerNorm, TensorNet init_norm / out_norm,
models/tensornet.py:232, 322), the Scalar head's last Linear fused with the per-molecule reduction
(tmdnet_dot_sum_*: output_modules.py:83-105 + model.py:263-283), and the copy-free stacked parameter rows
(kernels.stacked_rows == torch.cat).  First order in fp32 against fp64 autograd; second order (the
force-matching training step's double backward) against autograd of the composite."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.detach().double(), b.detach().double()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.mark.parametrize("C", [128, 384, 100])
def test_layer_norm_matches_composite(C):
    from torchmdnet import kernels
    g = torch.Generator(device=DEV).manual_seed(C)
    rows = 173
    x = (torch.randn(rows, C, device=DEV, generator=g) * 3 + 1).requires_grad_(True)
    w = torch.randn(C, device=DEV, generator=g).requires_grad_(True)
    b = torch.randn(C, device=DEV, generator=g).requires_grad_(True)
    y = kernels.layer_norm(x, w, b, 1e-5)
    xd, wd, bd = (t.detach().double().requires_grad_(True) for t in (x, w, b))
    yd = F.layer_norm(xd, (C,), wd, bd, 1e-5)
    assert _rel(y, yd) < 1e-5
    gy = torch.randn(rows, C, device=DEV, generator=g)
    gx, gw, gb = torch.autograd.grad(y, (x, w, b), gy, create_graph=True)
    gxd, gwd, gbd = torch.autograd.grad(yd, (xd, wd, bd), gy.double(), create_graph=True)
    for a_, b_ in ((gx, gxd), (gw, gwd), (gb, gbd)):
        assert _rel(a_, b_) < 1e-5
    # second order: a scalar of the first-order gradients, differentiated again
    s = (gx * gx.detach().sin()).sum() + (gw ** 2).sum()
    sd = (gxd * gx.detach().double().sin()).sum() + (gwd ** 2).sum()
    h = torch.autograd.grad(s, (x, w, b), allow_unused=True)
    hd = torch.autograd.grad(sd, (xd, wd, bd), allow_unused=True)
    for a_, b_ in zip(h, hd):
        if a_ is None or b_ is None:  # (no second-order path to the bias)
            assert (a_ if a_ is not None else b_ if b_ is not None else torch.zeros(1)).abs().max() == 0
            continue
        assert _rel(a_, b_) < 1e-4


def test_dot_sum_matches_composite():
    from torchmdnet import kernels
    g = torch.Generator(device=DEV).manual_seed(3)
    n, K, n_mol = 203, 64, 9
    batch = torch.sort(torch.randint(0, n_mol, (n,), device=DEV, generator=g)).values
    batch[-1] = n_mol - 1
    h = torch.randn(n, K, device=DEV, generator=g).requires_grad_(True)
    w = torch.randn(1, K, device=DEV, generator=g).requires_grad_(True)
    b0 = torch.randn(1, device=DEV, generator=g).requires_grad_(True)
    std, mean = torch.tensor([1.7], device=DEV), torch.tensor([-0.3], device=DEV)
    y = kernels.dot_sum(h, w, b0, batch, n_mol, std, mean)
    hd, wd, bd = (t.detach().double().requires_grad_(True) for t in (h, w, b0))
    yd = torch.zeros(n_mol, 1, dtype=torch.float64, device=DEV).index_add(0, batch, (hd @ wd.t() + bd) * 1.7) - 0.3
    assert _rel(y, yd) < 1e-6
    gy = torch.randn(n_mol, 1, device=DEV, generator=g)
    gh, gw, gb = torch.autograd.grad(y, (h, w, b0), gy, create_graph=True)
    ghd, gwd, gbd = torch.autograd.grad(yd, (hd, wd, bd), gy.double(), create_graph=True)
    for a_, b_ in ((gh, ghd), (gw, gwd), (gb, gbd)):
        assert _rel(a_, b_) < 1e-5
    s = (gh ** 2).sum() + (gw * 3).sum()
    sd = (ghd ** 2).sum() + (gwd * 3).sum()
    for a_, b_ in zip(torch.autograd.grad(s, (h, w), allow_unused=True),
                      torch.autograd.grad(sd, (hd, wd), allow_unused=True)):
        if b_ is None:
            continue
        assert _rel(a_, b_) < 1e-5


def test_stacked_rows_equals_cat():
    from torchmdnet import kernels
    torch.manual_seed(0)
    lins = [torch.nn.Linear(16, 8).to(DEV) for _ in range(3)]
    holder = {}
    x = torch.randn(5, 16, device=DEV)
    for step in range(2):  # the second call finds the parameters already stacked (no copy)
        W = kernels.stacked_rows(holder, "w", [m.weight for m in lins])
        assert torch.equal(W, torch.cat([m.weight for m in lins]))
        (x @ W.t()).pow(2).sum().backward()
    ref = [torch.autograd.grad((x @ torch.cat([m.weight for m in lins]).t()).pow(2).sum(), [m.weight for m in lins])]
    for m, r in zip(lins, ref[0]):
        assert torch.allclose(m.weight.grad, 2 * r, rtol=1e-5, atol=1e-6)
    assert holder["w"].data_ptr() == lins[0].weight.data_ptr()


def test_tensornet_scalar_head_fused_path_matches_unfused(monkeypatch):
    """The Scalar head's fused tail (mlp_act + dot_sum) against the module path (pre_reduce +
    fused_reduce) on a TensorNet model: energies, forces and force-loss parameter gradients."""
    from conftest import yaml_args
    from oracle import model_oracle as O
    from torchmdnet.models import output_modules
    from torchmdnet.models.model import create_model
    torch.manual_seed(0)
    m = create_model(yaml_args("tensornet", embedding_dimension=64, num_layers=2, num_rbf=32, derivative=True,
                               output_model="Scalar")).to(DEV)
    z, pos, batch = O.qm9_like(5)
    z, pos, batch = z.to(DEV), pos.float().to(DEV), batch.to(DEV)

    def run():
        m.zero_grad(set_to_none=True)
        y, f = m(z, pos.clone(), batch)
        ((y ** 2).sum() + (f ** 2).sum()).backward()
        return y.detach(), f.detach(), [p.grad.detach().clone() for p in m.parameters() if p.grad is not None]

    y1, f1, g1 = run()
    monkeypatch.setattr(output_modules.Scalar, "fused_head_reduce", lambda self, *a: None)
    y2, f2, g2 = run()
    assert _rel(y1, y2) < 1e-5 and _rel(f1, f2) < 1e-5
    assert len(g1) == len(g2)
    for a_, b_ in zip(g1, g2):
        assert _rel(a_, b_) < 1e-4
