"""TensorNet's hand-written second order (force-matching training; replaces autograd's double
differentiation of the PyTorch restatements, reference tensornet.py:287-410 under module.py:130-179):

* every node pass (tn_node.py, reference decompose_tensor / tensor_norm and the interaction's
  normalisation, product and residual, tensornet.py:47-67, 391-410) through
  ``tmdnet_tn_node_bwd2`` -- the same kernel code evaluated on dual numbers (forward-over-reverse);
* the channel mixes (``mix3``, tensornet.py:318-320, 354-356, 372-374) through GEMMs;
* the message (tensornet.py:329-332), bilinear in (edge factors, tensor), through its own forward and
  first-backward kernels;

each against ``tn_node._double_backward`` of the composite restatement in fp64 (1e-10), and the padded
C3 model's force-loss parameter gradients hip vs composite in fp32.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-300))


def _node_inputs(op, N, H, g):
    from torchmdnet import tn_node as T
    full = lambda: torch.randn(N, H, 3, 3, generator=g, dtype=torch.float64)  # noqa: E731
    comp = lambda: torch.randn(9, N, H, generator=g, dtype=torch.float64)  # noqa: E731
    if op == T.PRE or op == T.NORMS:
        return full(), None
    if op in (T.POST_O3, T.POST_SO3):
        return comp(), comp()
    if op == T.RESID:
        return full(), comp()
    if op == T.ENORM:
        return comp(), None
    return comp(), torch.randn(N, 3 * H, generator=g, dtype=torch.float64)  # EOUT


@pytest.mark.parametrize("op", list(range(7)), ids=["pre", "post_o3", "post_so3", "resid", "norms", "enorm", "eout"])
def test_node_pass_second_order_matches_composite(op):
    from torchmdnet import tn_node as T
    g = torch.Generator().manual_seed(op)
    N, H = 37, 24
    a, b = _node_inputs(op, N, H, g)
    out = T.op_composite(op, a, b)
    gout = torch.randn(out.shape, generator=g, dtype=torch.float64)
    ta = torch.randn(a.shape, generator=g, dtype=torch.float64)
    tb = None if b is None else torch.randn(b.shape, generator=g, dtype=torch.float64)
    prim = [a] if b is None else [a, b]
    fwd = (lambda x: T.op_composite(op, x)) if b is None else (lambda x, y: T.op_composite(op, x, y))
    ref = T._double_backward(fwd, prim, [gout], [ta] if b is None else [ta, tb])
    dv = lambda t: None if t is None else t.to(DEV)  # noqa: E731
    d_g = torch.empty(gout.shape, dtype=torch.float64, device=DEV)
    d_a = torch.empty(a.shape, dtype=torch.float64, device=DEV)
    d_b = None if b is None else torch.empty(b.shape, dtype=torch.float64, device=DEV)
    T.node_bwd2_launch(op, dv(a), dv(b), dv(gout), dv(ta), dv(tb), d_g, d_a, d_b)
    torch.cuda.synchronize()
    assert _rel(d_g.cpu(), ref[0]) < 1e-10
    assert _rel(d_a.cpu(), ref[1]) < 1e-10
    if b is not None:
        assert _rel(d_b.cpu(), ref[2]) < 1e-10


def test_mix3_second_order_matches_composite():
    from torchmdnet import tn_node as T
    g = torch.Generator().manual_seed(5)
    N, I, O = 53, 32, 48
    o = dict(dtype=torch.float64, device=DEV)
    c = torch.randn(9, N, I, generator=g, dtype=torch.float64).to(DEV)
    ws = [torch.randn(O, I, generator=g, dtype=torch.float64).to(DEV) for _ in range(3)]
    gout = torch.randn(9, N, O, generator=g, dtype=torch.float64).to(DEV)
    ggc = torch.randn(9, N, I, generator=g, dtype=torch.float64).to(DEV)
    for drop in (None, 1):  # a None weight cotangent too
        ggw = [None if i == drop else torch.randn(O, I, generator=g, dtype=torch.float64).to(DEV) for i in range(3)]
        got = T._mix3_second_order((False, True, True, True, True, True), gout, c, ws, ggc, ggw)
        ref = T._double_backward(T.mix3_composite, [c] + ws, [gout], [ggc] + ggw)
        for x, y in zip(got, ref):
            assert _rel(x, y) < 1e-10
    del o


def _tn_graph(n_mol=3):
    from torchmdnet.models.utils import OptimizedDistance
    g = torch.Generator().manual_seed(2)
    pos = (torch.randn(n_mol * 12, 3, generator=g, dtype=torch.float64) * 1.4).to(DEV)
    batch = torch.arange(n_mol).repeat_interleave(12).to(DEV)
    d = OptimizedDistance(0.0, 4.5, max_num_pairs=-64, return_vecs=True, loop=True)
    return d.graph(pos, batch)


def test_message_second_order_matches_composite(monkeypatch):
    from torchmdnet import kernels, tn_node
    graph = _tn_graph()
    g = torch.Generator().manual_seed(3)
    N, H, E = graph.n_nodes, 16, graph.n_edges
    ea = torch.randn(E, 3 * H, generator=g, dtype=torch.float64).to(DEV)
    Tc = torch.randn(9, N, H, generator=g, dtype=torch.float64).to(DEV)
    gmsg = torch.randn(9, N, H, generator=g, dtype=torch.float64).to(DEV)
    t_ea = torch.randn(E, 3 * H, generator=g, dtype=torch.float64).to(DEV)
    t_T = torch.randn(9, N, H, generator=g, dtype=torch.float64).to(DEV)
    # the kernels' precondition: edge factors -- and so their cotangents, functions of the pair distance
    # through the edge MLP -- are equal on the two directions of a pair (include/tmdnet.h)
    tr = graph.transpose.long()
    ea = 0.5 * (ea + ea[tr])
    t_ea = 0.5 * (t_ea + t_ea[tr])

    def second(mode):
        monkeypatch.setattr(tn_node, "SECOND_ORDER", mode)
        e, t, gm = (x.clone().requires_grad_(True) for x in (ea, Tc, gmsg))
        msg = kernels.tn_message(e, t, graph)
        first = torch.autograd.grad(msg, (e, t), gm, create_graph=True)
        return torch.autograd.grad(first, (gm, e, t), (t_ea, t_T))

    (g1, e1, t1), (g0, e0, t0) = second("hip"), second("composite")
    assert _rel(g1, g0) < 1e-10 and _rel(t1, t0) < 1e-10
    # the kernels number an edge factor's gradient by the row that reads it (the reverse of the
    # reference's scatter orientation); the two directions of a pair share one factor, so the per-pair
    # sums are what any consumer sees
    assert _rel(e1 + e1[tr], e0 + e0[tr]) < 1e-10


@pytest.mark.parametrize("layers,scaled", [(3, True), (2, False), (1, True)])
def test_mlp_second_order_matches_composite(layers, scaled, monkeypatch):
    """The Linear + SiLU stack (kernels.mlp_act: TensorNet's edge MLP 32 -> 128 -> 256 -> 384 times the cutoff,
    the embedding's 128 -> 256 -> 384, the output Linear) differentiated twice: the hand second order
    (kernels._mlp_second_order, tmdnet_mlp2_up / _down + hand GEMMs) vs autograd's double differentiation of
    the composite, fp32 (both) against each other at 1e-4 and the hand form against an fp64 composite."""
    from torchmdnet import kernels, tn_node
    g = torch.Generator(device=DEV).manual_seed(layers)
    dims = [32, 128, 256, 384][:layers + 1]
    M = 1000
    rn = lambda *sh: torch.randn(*sh, device=DEV, generator=g)  # noqa: E731
    x = rn(M, dims[0])
    sc = torch.rand(M, device=DEV, generator=g) if scaled else None
    ws = [rn(dims[i + 1], dims[i]) / dims[i] ** 0.5 for i in range(layers)]
    bs = [0.1 * rn(dims[i + 1]) for i in range(layers)]
    gy = rn(M, dims[-1])
    prim = [x] + ([sc] if scaled else []) + ws + bs
    tang = [rn(*t.shape) for t in prim]

    def second(mode, dtype):
        monkeypatch.setattr(tn_node, "SECOND_ORDER", mode)
        xs = [t.to(dtype).clone().requires_grad_(True) for t in prim]
        g0 = gy.to(dtype).clone().requires_grad_(True)
        xx, rest = xs[0], xs[1:]
        s_ = rest[0] if scaled else None
        wb = rest[1:] if scaled else rest
        if dtype == torch.float64:
            y = kernels._mlp_composite(xx, s_, *wb)
        else:
            y = kernels.mlp_act(xx, list(wb[:layers]), list(wb[layers:]), torch.nn.SiLU(), s_)
        first = torch.autograd.grad(y, xs, g0, create_graph=True)
        return torch.autograd.grad(first, xs + [g0], [t.to(dtype) for t in tang], allow_unused=True)

    hip, comp, ref = second("hip", torch.float32), second("composite", torch.float32), second("composite", torch.float64)
    for a, b, r in zip(hip, comp, ref):
        assert (a is None) == (r is None)
        if a is None:
            continue
        assert _rel(a.double(), r) < 1e-4
        assert _rel(a, b) < 1e-4


@pytest.mark.parametrize("C", [128, 384])
def test_layer_norm_second_order_matches_composite(C, monkeypatch):
    """TensorNet's LayerNorms (init_norm C = H, out_norm C = 3H) differentiated twice: the hand second order
    (tmdnet_layernorm_bwd2_f32) vs autograd's double differentiation of the composite (fp32 and fp64)."""
    from torchmdnet import kernels, tn_node
    g = torch.Generator(device=DEV).manual_seed(C)
    M = 300
    rn = lambda *sh: torch.randn(*sh, device=DEV, generator=g)  # noqa: E731
    x, w, b, gy = rn(M, C) * 2 + 0.5, rn(C), rn(C), rn(M, C)
    tang = [rn(M, C), rn(C), rn(C)]

    def second(mode, dtype):
        monkeypatch.setattr(tn_node, "SECOND_ORDER", mode)
        xs = [t.to(dtype).clone().requires_grad_(True) for t in (x, w, b)]
        g0 = gy.to(dtype).clone().requires_grad_(True)
        y = kernels._ln_composite(*xs, 1e-5) if dtype == torch.float64 else kernels.layer_norm(*xs, 1e-5)
        first = torch.autograd.grad(y, xs, g0, create_graph=True)
        return torch.autograd.grad(first, xs[:2] + [g0], [t.to(dtype) for t in tang], allow_unused=True)

    hip, comp, ref = second("hip", torch.float32), second("composite", torch.float32), second("composite", torch.float64)
    for a, bb, r in zip(hip, comp, ref):
        assert _rel(a.double(), r) < 1e-4
        assert _rel(a, bb) < 1e-4


@pytest.mark.parametrize("n_atoms", [168, 5000])
def test_dot_sum_second_order_matches_composite(n_atoms):
    """The Scalar head's last Linear fused with the molecule sum (kernels.dot_sum) differentiated twice: the hand
    VJP of its first backward (dot-sum / TN launches, no library GEMM) vs the composite differentiated twice
    in fp64, every input (h, w, b0) and the seed gy."""
    from torchmdnet import kernels
    g = torch.Generator(device=DEV).manual_seed(n_atoms)
    H, n_mol = 64, 8
    rn = lambda *sh: torch.randn(*sh, device=DEV, generator=g)  # noqa: E731
    batch = torch.sort(torch.randint(0, n_mol, (n_atoms,), device=DEV, generator=g)).values
    batch[:n_mol] = torch.arange(n_mol, device=DEV)
    batch = torch.sort(batch).values
    h, w, b0, gy = rn(n_atoms, H), rn(H), rn(1), rn(n_mol, 1)
    std, mean = torch.scalar_tensor(1.7, device=DEV), torch.scalar_tensor(0.3, device=DEV)
    tang = [rn(n_atoms, H), rn(H), rn(1)]

    def second(dtype):
        xs = [t.to(dtype).clone().requires_grad_(True) for t in (h, w, b0)]
        g0 = gy.to(dtype).clone().requires_grad_(True)
        s, m = std.to(dtype), mean.to(dtype)
        if dtype == torch.float64:
            y = kernels._dot_sum_composite(xs[0], xs[1], xs[2], batch, n_mol, s, m)
        else:
            y = kernels.dot_sum(xs[0], xs[1], xs[2], batch, n_mol, s, m)
        first = torch.autograd.grad(y, xs, g0, create_graph=True)
        return torch.autograd.grad(first, xs[:2] + [g0], [t.to(dtype) for t in tang], allow_unused=True)

    hip, ref = second(torch.float32), second(torch.float64)
    for a, r in zip(hip, ref):
        assert _rel(a.double().reshape(r.shape), r) < 1e-5


def test_embedding_second_order_matches_composite(monkeypatch):
    """TensorEmbedding's aggregation (tensornet.py:295-315) differentiated twice: the hand second order
    (tmdnet_tn_embed_bwd2: the first-order kernels on dual numbers) vs autograd's double differentiation of
    the composite, fp64.  Inputs and tangents obey the kernels' pair precondition: W, C (and their tangents)
    equal on the two directions of a pair, u (and its tangent) opposite -- as in the model, where they are
    functions of the pair distance / the displacement."""
    from torchmdnet import kernels, tn_node
    graph = _tn_graph()
    g = torch.Generator().manual_seed(4)
    N, H, E = graph.n_nodes, 16, graph.n_edges
    rn = lambda *s: torch.randn(*s, generator=g, dtype=torch.float64).to(DEV)  # noqa: E731
    tr = graph.transpose.long()
    sym = lambda t: 0.5 * (t + t[tr])  # noqa: E731
    asym = lambda t: 0.5 * (t - t[tr])  # noqa: E731
    P, Q, W, C, u, gE = rn(N, H), rn(N, H), sym(rn(E, 3 * H)), sym(rn(E)), asym(rn(E, 3)), rn(9, N, H)
    tP, tQ, tW, tC, tu = rn(N, H), rn(N, H), sym(rn(E, 3 * H)), sym(rn(E)), asym(rn(E, 3))

    def second(mode):
        monkeypatch.setattr(tn_node, "SECOND_ORDER", mode)
        xs = [x.clone().requires_grad_(True) for x in (P, Q, W, C, u, gE)]
        out = kernels.tn_embed(*xs[:5], graph)
        first = torch.autograd.grad(out, xs[:5], xs[5], create_graph=True)
        return torch.autograd.grad(first, xs, (tP, tQ, tW, tC, tu))

    a, b = second("hip"), second("composite")
    assert _rel(a[0], b[0]) < 1e-10 and _rel(a[1], b[1]) < 1e-10  # P, Q
    assert _rel(a[5], b[5]) < 1e-10  # gE
    # per-edge rows are numbered by the row that reads them: compare what any consumer sees, the pair sums
    # (W, C: symmetric) and differences (u: antisymmetric)
    assert _rel(a[2] + a[2][tr], b[2] + b[2][tr]) < 1e-10
    assert _rel(a[3] + a[3][tr], b[3] + b[3][tr]) < 1e-10
    assert _rel(a[4] - a[4][tr], b[4] - b[4][tr]) < 1e-10


@pytest.mark.parametrize("static_shapes", [True, False])
def test_tensornet_force_loss_gradients_hip_vs_composite(static_shapes, monkeypatch):
    """C3-shaped TensorNet (O(3)) force-matching loss: parameter gradients through the hand second order
    equal those through the composite restatements (fp32)."""
    import os
    import yaml
    from conftest import GOLDEN
    from torchmdnet import tn_node
    from torchmdnet.models.model import create_model
    with open(os.path.join(GOLDEN, "configs", "tensornet_rmd17.yaml")) as fh:
        args = yaml.safe_load(fh)
    args.update(prior_model=None, precision=32, derivative=True, static_shapes=static_shapes)
    torch.manual_seed(0)
    m = create_model(args).to(DEV)
    g = torch.Generator().manual_seed(1)
    z = torch.tensor([6] * 9 + [1] * 8 + [8] * 4, dtype=torch.long).repeat(4).to(DEV)
    pos = (torch.randn(z.shape[0], 3, generator=g) * 1.6).to(DEV)
    batch = torch.arange(4).repeat_interleave(21).to(DEV)

    def grads(mode):
        monkeypatch.setattr(tn_node, "SECOND_ORDER", mode)
        m.zero_grad(set_to_none=True)
        y, f = m(z, pos, batch)
        (y.pow(2).sum() + f.pow(2).sum()).backward()
        return {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}

    a, b = grads("hip"), grads("composite")
    assert a.keys() == b.keys()
    for n in a:
        assert _rel(a[n], b[n]) < 2e-5, n
