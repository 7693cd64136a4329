"""The ET message kernels with every activation of the reference's act_class_mapping
(models/utils.py:579-584) for the dk/dv projections (`activation`) and the attention
(`attn_activation`, torchmd_et.py:316): tmdnet_et_message_fwd / _bwd / _bwd2 with TMDNET_ET_ACT flags
against autograd over the plain restatement (kernels.et_message_composite), fp64."""
import pytest
import torch

from oracle import model_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
NAMES = ["silu", "ssp", "tanh", "sigmoid"]


def _setup(H=32, heads=4, seed=0):
    from torchmdnet import kernels
    torch.manual_seed(seed)
    z, pos, batch = O.qm9_like(2)
    pos = pos.to(DEV)
    g = kernels.build_graph(pos, batch.to(DEV), 0.0, 5.0, 64 * pos.shape[0], loop=True)
    N, E = pos.shape[0], g.n_edges
    o = dict(dtype=torch.float64, device=DEV)
    T = g.transpose.long()
    sym = lambda t: ((t + t[T]) / 2).detach().requires_grad_(True)  # noqa: E731  (functions of |r|)
    q, k = torch.randn(N, H, **o).requires_grad_(True), torch.randn(N, H, **o).requires_grad_(True)
    v = torch.randn(N, 3 * H, **o).requires_grad_(True)
    vec = torch.randn(N, 3, H, **o).requires_grad_(True)
    pk, pv, C = sym(torch.randn(E, H, **o)), sym(torch.randn(E, 3 * H, **o)), sym(torch.rand(E, **o))
    r = g.distances.detach()
    u = (g.deltas.detach() / torch.where(r > 0, r, torch.ones_like(r)).unsqueeze(1)).requires_grad_(True)
    return g, heads, T, (q, k, v, vec, pk, pv, C, u)


@pytest.mark.parametrize("act_kv", NAMES)
@pytest.mark.parametrize("act_at", NAMES)
def test_message_activations_first_order(act_kv, act_at):
    from torchmdnet import kernels
    acts = kernels.et_act_flags(NAMES.index(act_kv), NAMES.index(act_at))
    g, heads, T, ins = _setup()
    N = ins[0].shape[0]
    xo, vo = kernels.et_message(*ins, g, heads, acts)
    xr, vr = kernels.et_message_composite(*ins, g.src.long(), g.dst.long(), N, heads, acts)
    assert torch.allclose(xo, xr, atol=1e-11) and torch.allclose(vo, vr, atol=1e-11)
    gx, gv = torch.randn_like(xo), torch.randn_like(vo)
    a = torch.autograd.grad((xo, vo), ins, (gx, gv))
    b = torch.autograd.grad((xr, vr), ins, (gx, gv))
    for name, ga, gb in zip("q k v vec pk pv C u".split(), a, b):
        if name in ("pk", "pv", "C"):  # per-edge gradients of symmetric inputs: symmetrised sums
            ga, gb = ga + ga[T], gb + gb[T]
        if name == "u":
            ga, gb = ga - ga[T], gb - gb[T]
        assert torch.allclose(ga, gb, atol=1e-10, rtol=1e-9), name


@pytest.mark.parametrize("act_kv,act_at", [("ssp", "tanh"), ("tanh", "sigmoid"), ("sigmoid", "ssp"),
                                           ("silu", "tanh")])
def test_message_activations_second_order(act_kv, act_at):
    """tmdnet_et_message_bwd2 (the force-loss second order) with the activation codes."""
    from torchmdnet import kernels
    acts = kernels.et_act_flags(NAMES.index(act_kv), NAMES.index(act_at))
    g, heads, T, prim = _setup(seed=1)
    q, k, v, vec, pk, pv, C, u = prim
    N, H = q.shape
    o = dict(dtype=torch.float64, device=DEV)
    gx, gvec = torch.randn(N, H, **o).requires_grad_(True), torch.randn(N, 3, H, **o).requires_grad_(True)
    ins = [gx, gvec, q, k, v, vec, pk, pv, C, u]
    outs = kernels._ETMessageBwd.apply(gx, gvec, q, k, v, vec, pk, pv, C, u, g, heads, acts)
    outs = [t for t in outs if t.numel()]
    gg = [torch.randn_like(t) for t in outs]
    a = torch.autograd.grad(outs, ins, gg, allow_unused=True)
    xo, vo = kernels.et_message_composite(q, k, v, vec, pk, pv, C, u, g.src.long(), g.dst.long(), N, heads, acts)
    first = torch.autograd.grad((xo, vo), list(prim), (gx, gvec), create_graph=True)
    b = torch.autograd.grad(first, ins, gg, allow_unused=True)
    for n, ga, gb in zip("gx gvec q k v vec pk pv C u".split(), a, b):
        gb = torch.zeros_like(ga) if gb is None else gb
        assert torch.allclose(ga, gb, atol=1e-10, rtol=1e-8), n


def test_message_rejects_unknown_activation_code():
    from torchmdnet import kernels
    g, heads, T, ins = _setup()
    with pytest.raises(RuntimeError):
        kernels.et_message(*ins, g, heads, kernels.et_act_flags(7, 0))
