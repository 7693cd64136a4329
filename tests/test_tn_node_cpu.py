"""CPU checks of the TensorNet compact-layout node algebra (torchmdnet/tn_node.py) and of the TN
modules' orchestration around the HIP launches.

(1) The compact basis and every fused pass's PyTorch composite against the reference's own
    full-layout formulation (models/tensornet.py:16-67, 316-326, 391-410), values and gradients.
(2) TensorEmbedding / Interaction run on CPU with the native launches (tn_embed, tn_message, the
    node passes) replaced, in this test only, by emulations built from those composites; compared
    with the reference math in the [N, H, 3, 3] layout (restated here as in oracle/model_oracle.py):
    outputs, first-order gradients and the double backward.  The HIP kernels themselves are
    checked against the same composites on the GPU (test_gpu_parity.py).
"""
import math

import pytest
import torch

from torchmdnet import _native as nat
from torchmdnet import kernels, tn_node
from torchmdnet.models.tensornet import Interaction, TensorEmbedding

DT = torch.float64


# ----------------------------------------------------------------------------- reference math
def _decompose(t):
    eye = torch.eye(3, dtype=t.dtype)
    i = t.diagonal(dim1=-2, dim2=-1).mean(-1)[..., None, None] * eye
    return i, 0.5 * (t - t.transpose(-2, -1)), 0.5 * (t + t.transpose(-2, -1)) - i


def _tnorm(t):
    return (t ** 2).sum((-2, -1))


def _skew(v):
    z = torch.zeros_like(v[:, 0])
    return torch.stack((z, -v[:, 2], v[:, 1], v[:, 2], z, -v[:, 0], -v[:, 1], v[:, 0], z), dim=1).view(-1, 3, 3)


def _sym(v):
    t = v.unsqueeze(-1) * v.unsqueeze(-2)
    i = t.diagonal(dim1=-2, dim2=-1).mean(-1)[..., None, None] * torch.eye(3, dtype=v.dtype)
    return 0.5 * (t + t.transpose(-2, -1)) - i


def _chan(lin, t):
    return lin(t.permute(0, 2, 3, 1)).permute(0, 3, 1, 2)


def ref_embedding(mod, z, src, dst, C, u, f):
    """tensornet.py:287-326 (scatter to edge_index[0] = src, gather edge_index[1] = dst)."""
    N, H = z.shape[0], mod.hidden_channels
    W1 = mod.distance_proj1(f) * C[:, None]
    W2 = mod.distance_proj2(f) * C[:, None]
    W3 = mod.distance_proj3(f) * C[:, None]
    Z = mod.emb(z)
    Zij = mod.emb2(torch.cat([Z[src], Z[dst]], dim=1))[..., None, None]
    eye = torch.eye(3, dtype=DT)
    zero = torch.zeros(N, H, 3, 3, dtype=DT)
    I = zero.index_add(0, src, Zij * W1[..., None, None] * eye)
    A = zero.index_add(0, src, Zij * W2[..., None, None] * _skew(u)[:, None])
    S = zero.index_add(0, src, Zij * W3[..., None, None] * _sym(u)[:, None])
    norm = mod.init_norm(_tnorm(I + A + S))
    I, A, S = (_chan(mod.linears_tensor[k], t) for k, t in enumerate((I, A, S)))
    for ls in mod.linears_scalar:
        norm = mod.act(ls(norm))
    norm = norm.reshape(N, H, 3)
    return I * norm[..., 0, None, None] + A * norm[..., 1, None, None] + S * norm[..., 2, None, None]


def ref_interaction_out(mod, X, src, dst, C, f):
    """tensornet.py:383-410."""
    N, H = X.shape[0], X.shape[1]
    ea = f
    for ls in mod.linears_scalar:
        ea = mod.act(ls(ea))
    ea = (ea * C[:, None]).reshape(-1, H, 3)
    Xn = X / (_tnorm(X) + 1)[..., None, None]
    I, A, S = _decompose(Xn)
    I, A, S = (_chan(mod.linears_tensor[k], t) for k, t in enumerate((I, A, S)))
    Y = I + A + S
    zero = torch.zeros(N, H, 3, 3, dtype=DT)
    msg = zero.index_add(0, src, ea[..., 0, None, None] * I[dst]) \
        + zero.index_add(0, src, ea[..., 1, None, None] * A[dst]) \
        + zero.index_add(0, src, ea[..., 2, None, None] * S[dst])
    if mod.equivariance_invariance_group == "O(3)":
        I, A, S = _decompose(torch.matmul(msg, Y) + torch.matmul(Y, msg))
    else:
        I, A, S = _decompose(2 * torch.matmul(Y, msg))
    normp1 = (_tnorm(I + A + S) + 1)[..., None, None]
    I, A, S = I / normp1, A / normp1, S / normp1
    I, A, S = (_chan(mod.linears_tensor[3 + k], t) for k, t in enumerate((I, A, S)))
    dX = I + A + S
    return Xn + dX + torch.matmul(dX, dX)  # the reference reassigns X = X / (|X|^2 + 1) (:391)


# ----------------------------------------------------------------------------- emulation
def _fake_node_fwd(op, a, b, out):
    out.copy_(tn_node.op_composite(op, a, b))


def _vjp(fn, ins, gout):
    with torch.enable_grad():
        leaves = [None if t is None else t.detach().clone().requires_grad_(True) for t in ins]
        out = fn(*leaves)
        live = [t for t in leaves if t is not None]
        g = torch.autograd.grad(out, live, gout, allow_unused=True)
    it = iter(g)
    return [None if t is None else next(it) for t in leaves]


def _fake_node_bwd(op, a, b, gout, gadd, ga, gb):
    g = _vjp(lambda x, y=None: tn_node.op_composite(op, x, y), [a, b], gout)
    if ga is not None:
        ga.copy_(g[0] + (0 if gadd is None else gadd))
    if gb is not None:
        gb.copy_(g[1])


def _fake_embed_fwd(P, Q, W, C, u, graph, out):
    out.copy_(kernels.tn_embed_composite(P, Q, W, C, u, graph))


def _fake_embed_bwd(P, Q, W, C, u, graph, gE, gP, gQ, gW, gC, gu):
    g = _vjp(lambda *t: kernels.tn_embed_composite(*t, graph), [P, Q, W, C, u], gE)
    for dst, src in zip((gP, gQ, gW, gC, gu), g):
        dst.copy_(src)


def _fake_msg_fwd(ea, Tc, graph, out, pairs=None):
    out.copy_(kernels.tn_message_composite(kernels._ea_edges(ea, pairs), Tc, graph))


def _fake_msg_bwd(ea, Tc, graph, gmsg, gea, gT, gadd=None, pairs=None):
    g = _vjp(lambda e, t: kernels.tn_message_composite(kernels._ea_edges(e, pairs), t, graph), [ea, Tc], gmsg)
    gea.copy_(g[0])
    gT.copy_(g[1] + (0 if gadd is None else gadd))


@pytest.fixture
def emulated(monkeypatch):
    monkeypatch.setattr(tn_node, "node_fwd_launch", _fake_node_fwd)
    monkeypatch.setattr(tn_node, "node_bwd_launch", _fake_node_bwd)
    monkeypatch.setattr(kernels, "tn_embed_fwd_launch", _fake_embed_fwd)
    monkeypatch.setattr(kernels, "tn_embed_bwd_launch", _fake_embed_bwd)
    monkeypatch.setattr(kernels, "tn_message_fwd_launch", _fake_msg_fwd)
    monkeypatch.setattr(kernels, "tn_message_bwd_launch", _fake_msg_bwd)
    monkeypatch.setattr(nat, "require_gpu", lambda t, what: None)


def _system(seed=0, cutoff=4.0):
    g = torch.Generator().manual_seed(seed)
    sizes = [5, 7, 4]
    pos = torch.cat([torch.randn(s, 3, generator=g, dtype=DT) * 1.3 for s in sizes])
    batch = torch.cat([torch.full((s,), i, dtype=torch.long) for i, s in enumerate(sizes)])
    d = (pos[:, None] - pos[None]).norm(dim=-1)
    adj = (d < cutoff) & (batch[:, None] == batch[None])
    ei = adj.nonzero().t().contiguous()
    graph, perm = kernels.EdgeGraph.from_edge_index(ei, pos.shape[0])
    ei = ei[:, perm]
    vecs = pos[ei[0]] - pos[ei[1]]
    r = vecs.norm(dim=-1)
    u = torch.where((r > 0)[:, None], vecs / torch.where(r > 0, r, torch.ones_like(r))[:, None], vecs)
    C = 0.5 * (torch.cos(r * math.pi / cutoff) + 1.0)
    return pos.shape[0], ei, graph, r, u, C


def _feat(r, R):
    mu = torch.linspace(0, 4, R, dtype=DT)
    return torch.exp(-((r[:, None] - mu) ** 2))


def _perturb(mod, seed):
    torch.manual_seed(seed)
    with torch.no_grad():
        for p in mod.parameters():
            p.add_(0.1 * torch.randn_like(p))
    return mod


# ----------------------------------------------------------------------------- (1) composites
def test_compact_basis_roundtrip():
    torch.manual_seed(0)
    X = torch.randn(4, 6, 3, 3, dtype=DT)
    c = tn_node.decomp9(X)
    assert torch.allclose(tn_node.full9(c), X, atol=1e-14)  # I + A + S == X
    I, A, S = _decompose(X)
    assert torch.allclose(tn_node.full9(torch.cat([c[:1], torch.zeros_like(c[1:])])), I)
    assert torch.allclose(tn_node.full9(torch.cat([torch.zeros_like(c[:1]), c[1:4], torch.zeros_like(c[4:])])), A)
    assert torch.allclose(tn_node.full9(torch.cat([torch.zeros_like(c[:4]), c[4:]])), S)
    assert torch.allclose(tn_node.decomp9(tn_node.full9(c)), c, atol=1e-14)


@pytest.mark.parametrize("op", ["pre", "post_o3", "post_so3", "resid", "norms", "enorm", "eout"])
def test_op_composites_match_reference_formulation(op):
    torch.manual_seed(1)
    N, H = 5, 4
    X = torch.randn(N, H, 3, 3, dtype=DT, requires_grad=True)
    a = torch.randn(9, N, H, dtype=DT, requires_grad=True)
    b = torch.randn(9, N, H, dtype=DT, requires_grad=True)
    f = torch.randn(N, 3 * H, dtype=DT, requires_grad=True)
    mm = torch.matmul
    if op == "pre":
        ins, mine = (X,), tn_node.op_composite(tn_node.PRE, X)
        Xn = X / (_tnorm(X) + 1)[..., None, None]
        ref = tn_node.decomp9(sum(_decompose(Xn)))
    elif op in ("post_o3", "post_so3"):
        code = tn_node.POST_O3 if op == "post_o3" else tn_node.POST_SO3
        ins, mine = (a, b), tn_node.op_composite(code, a, b)
        Y, M = tn_node.full9(a), tn_node.full9(b)
        I, A, S = _decompose(mm(M, Y) + mm(Y, M) if op == "post_o3" else 2 * mm(Y, M))
        n = (_tnorm(I + A + S) + 1)[..., None, None]
        ref = tn_node.decomp9(I / n + A / n + S / n)
    elif op == "resid":
        ins, mine = (X, b), tn_node.op_composite(tn_node.RESID, X, b)
        D = tn_node.full9(b)
        ref = X / (_tnorm(X) + 1)[..., None, None] + D + mm(D, D)
    elif op == "norms":
        ins, mine = (X,), tn_node.op_composite(tn_node.NORMS, X)
        I, A, S = _decompose(X)
        ref = torch.cat((_tnorm(I), _tnorm(A), _tnorm(S)), dim=-1)
    elif op == "enorm":
        ins, mine = (a,), tn_node.op_composite(tn_node.ENORM, a)
        ref = _tnorm(tn_node.full9(a))
    else:
        ins, mine = (a, f), tn_node.op_composite(tn_node.EOUT, a, f)
        nr = f.reshape(N, H, 3)
        I = tn_node.full9(torch.cat([a[:1], torch.zeros_like(a[1:])]))
        A = tn_node.full9(torch.cat([torch.zeros_like(a[:1]), a[1:4], torch.zeros_like(a[4:])]))
        S = tn_node.full9(torch.cat([torch.zeros_like(a[:4]), a[4:]]))
        ref = I * nr[..., 0, None, None] + A * nr[..., 1, None, None] + S * nr[..., 2, None, None]
    assert torch.allclose(mine, ref, rtol=1e-12, atol=1e-12)
    g = torch.randn_like(ref)
    g1 = torch.autograd.grad(mine, ins, g)
    g2 = torch.autograd.grad(ref, ins, g)
    for x, y in zip(g1, g2):
        assert torch.allclose(x, y, rtol=1e-11, atol=1e-11)


def test_mix3_matches_channel_linear():
    torch.manual_seed(2)
    N, H = 5, 6
    lins = [torch.nn.Linear(H, H, bias=False, dtype=DT) for _ in range(3)]
    X = torch.randn(N, H, 3, 3, dtype=DT)
    c = tn_node.decomp9(X)
    out = tn_node.mix3_composite(c, *(l.weight for l in lins))
    I, A, S = _decompose(X)
    ref = sum(_chan(l, t) for l, t in zip(lins, (I, A, S)))
    assert torch.allclose(tn_node.full9(out), ref, atol=1e-12)


# ----------------------------------------------------------------------------- (2) modules
@pytest.mark.parametrize("static_mult", [1.0, 3.0])
def test_embedding_matches_reference(emulated, static_mult):
    n, ei, graph, r, u, C = _system()
    graph.self0_mult = static_mult
    H, R = 8, 6
    f = _feat(r, R).requires_grad_(True)
    u = u.clone().requires_grad_(True)
    C = C.clone().requires_grad_(True)
    torch.manual_seed(3)
    mod = _perturb(TensorEmbedding(H, R, torch.nn.SiLU, 0.0, 4.0, dtype=DT).to(DT), 4)
    z = torch.randint(1, 10, (n,))
    graph.cutoff = C
    mine = mod(z, graph, r, u, f)
    # static_shapes multiplicity: atom 0's self loop counted static_mult times
    src, dst = ei[0], ei[1]
    extra = int(static_mult) - 1
    self0 = ((src == 0) & (dst == 0)).nonzero().flatten()
    idx = torch.cat([torch.arange(src.numel())] + [self0] * extra)
    ref = ref_embedding(mod, z, src[idx], dst[idx], C[idx], u[idx], f[idx])
    assert torch.allclose(mine, ref, rtol=1e-10, atol=1e-10)
    g = torch.randn_like(ref)
    params = list(mod.parameters())
    g1 = torch.autograd.grad(mine, [f, u, C] + params, g, allow_unused=True)
    g2 = torch.autograd.grad(ref, [f, u, C] + params, g, allow_unused=True)
    for x, y in zip(g1, g2):
        if y is None:
            assert x is None or x.abs().max() == 0
            continue
        assert torch.allclose(x, y, rtol=1e-9, atol=1e-10)


@pytest.mark.parametrize("group", ["O(3)", "SO(3)"])
def test_interaction_matches_reference_incl_double_backward(emulated, group):
    n, ei, graph, r, u, C = _system(seed=1)
    H, R = 8, 6
    f = _feat(r, R).requires_grad_(True)
    C = C.clone().requires_grad_(True)
    graph.cutoff = C
    torch.manual_seed(5)
    mod = _perturb(Interaction(R, H, torch.nn.SiLU, 0.0, 4.0, group, DT).to(DT), 6)
    X = (0.5 * torch.randn(n, H, 3, 3, dtype=DT)).requires_grad_(True)
    mine = mod(X, graph, r, f)
    ref = ref_interaction_out(mod, X, ei[0], ei[1], C, f)
    assert torch.allclose(mine, ref, rtol=1e-10, atol=1e-10)
    params = list(mod.parameters())
    g = torch.randn_like(ref)
    # first order (with graph) and a second-order functional of it, as force-loss training does
    g1 = torch.autograd.grad(mine, [X, f, C], g, create_graph=True)
    g2 = torch.autograd.grad(ref, [X, f, C], g, create_graph=True)
    for x, y in zip(g1, g2):
        assert torch.allclose(x, y, rtol=1e-9, atol=1e-10)
    l1 = sum((x ** 2).sum() for x in g1)
    l2 = sum((y ** 2).sum() for y in g2)
    h1 = torch.autograd.grad(l1, [X, f] + params, allow_unused=True)
    h2 = torch.autograd.grad(l2, [X, f] + params, allow_unused=True)
    for x, y in zip(h1, h2):
        assert (x is None) == (y is None)
        if x is not None:
            assert torch.allclose(x, y, rtol=1e-8, atol=1e-9)


# ----------------------------------------------------------------------------- (3) whole model
def _cpu_graph(self, pos, batch=None):
    """Brute-force symmetric CSR graph on the CPU with autograd-carrying deltas / distances (test
    emulation of tmdnet_nl_build; the reference CPU op's pair set, neighbors_cpu.cpp:24-95)."""
    n = pos.shape[0]
    if batch is None:
        batch = torch.zeros(n, dtype=torch.long)
    d = (pos[:, None] - pos[None]).norm(dim=-1)
    adj = (d < self.cutoff_upper) & (d >= self.cutoff_lower) & (batch[:, None] == batch[None])
    adj.fill_diagonal_(False)
    adj |= torch.eye(n, dtype=torch.bool)
    ei = adj.nonzero().t().contiguous()
    graph, perm = kernels.EdgeGraph.from_edge_index(ei, n)
    ei = ei[:, perm]
    graph.deltas = pos[ei[0]] - pos[ei[1]]
    sq = (graph.deltas ** 2).sum(1)
    self_e = ei[0] == ei[1]
    graph.distances = torch.where(self_e, torch.zeros_like(sq), torch.where(self_e, torch.ones_like(sq), sq).sqrt())
    return graph


def _cpu_edge_geometry(graph, mu, beta, cutoff_lower, cutoff_upper, rbf_type, want=(True, True, True), rows=None,
                       fan=(1, 1)):
    f, C, u = kernels._edge_geom_composite(graph.deltas, graph.distances, graph.src == graph.dst, mu, beta,
                                           float(cutoff_lower), float(cutoff_upper), rbf_type, want)
    if tuple(fan) != (1, 1):  # one alias per consumer, as the HIP path returns them
        return [f] * fan[0], [C] * fan[1], u
    return f, C, u


@pytest.mark.parametrize("name", ["tn_tiny_o3_static_f64", "tn_tiny_so3_dyn_f64"])
def test_tensornet_model_emulated_matches_reference_fixture(emulated, monkeypatch, name):
    """TorchMD_Net(TensorNet) end to end on the CPU with every native launch emulated (neighbour list
    and edge geometry included) against the reference fixture: energies, forces and the
    force-loss parameter gradients (double backward)."""
    import numpy as np
    from conftest import golden, state_dict_from, yaml_args
    from torchmdnet.models.model import create_model
    from torchmdnet.models.utils import OptimizedDistance
    monkeypatch.setattr(OptimizedDistance, "graph", _cpu_graph)
    monkeypatch.setattr(kernels, "edge_geometry", _cpu_edge_geometry)
    d = golden(name + ".npz")
    args = yaml_args("tensornet", embedding_dimension=32, num_layers=2, num_rbf=16, max_num_neighbors=32,
                     cutoff_upper=4.5, derivative=True, output_model="Scalar", precision=64,
                     equivariance_invariance_group="SO(3)" if "so3" in name else "O(3)")
    m = create_model(args)
    m.load_state_dict({k: torch.tensor(v) for k, v in state_dict_from(d).items()})
    m.representation_model.static_shapes = "static" in name
    y, neg_dy = m(torch.tensor(d["z"]), torch.tensor(d["pos"]), torch.tensor(d["batch"]))
    rel = lambda a, b: float(np.abs(a.detach().numpy() - b).max() / np.abs(b).max())
    assert rel(y, d["y"]) < 1e-9
    assert rel(neg_dy, d["neg_dy"]) < 1e-9
    loss = (y ** 2).sum() + (neg_dy ** 2).sum()
    named = [(n, p) for n, p in m.named_parameters() if p.requires_grad]
    grads = torch.autograd.grad(loss, [p for _, p in named], allow_unused=True)
    for (n, _), g in zip(named, grads):
        ref = d["g2/" + n]
        got = np.zeros_like(ref) if g is None else g.detach().numpy()
        assert np.allclose(got, ref, rtol=1e-6, atol=1e-8), n
