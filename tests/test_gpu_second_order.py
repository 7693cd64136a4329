"""GPU checks of the hand-scheduled ET second order (et_stack._second_order).

* ``tmdnet_et_adjoint_epi_ln`` (fused epilogue-backward VJP + LayerNorm-backward VJP) against its
  restatement ``epi_adjoint`` / ``ln_adjoint`` (themselves checked against double autograd on CPU,
  tests/test_et_stack_cpu.py), fp64 1e-12 and fp32 1e-5, with and without the vec terms / LayerNorm;
* the force-matching weight gradients of the real model (HIP kernels end to end) with the hand
  second order against TMDNET's composite second order (autograd over the recomputed stack), fp64,
  with and without the fused out_norm and dr mode.
"""
import pytest
import torch

from conftest import yaml_args
from oracle import model_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.mark.parametrize("dtype,tol", [(torch.float64, 1e-12), (torch.float32, 2e-5)])
@pytest.mark.parametrize("with_vec", [True, False])
@pytest.mark.parametrize("with_epi,with_ln", [(True, True), (True, False), (False, True)])
@pytest.mark.parametrize("split_vec", [False, True])  # the vec cotangent as two addends (..._ln2)
def test_adjoint_epi_ln_kernel(dtype, tol, with_vec, with_epi, with_ln, split_vec):
    from torchmdnet import et_stack as ES
    torch.manual_seed(0)
    N, H = 77, 128
    r = lambda *s: torch.randn(*s, device=DEV, dtype=dtype)  # noqa: E731
    epi = None
    if with_epi:
        epi = (r(N, 3 * H), r(N, 3, 3 * H) if with_vec else None, r(N, H), r(N, 3, H) if with_vec else None,
               r(N, 3, 3 * H) if with_vec else None, r(N, 3 * H))
    ln = None
    if with_ln:
        x = r(N, H) * 2 + 0.3
        _, mean, rstd = torch.native_layer_norm(x, [H], None, None, 1e-5)
        ln = (x, mean, rstd, r(H), r(N, H))
    gbx, gbv = r(N, H), (r(N, 3, H) if with_vec else None)
    if split_vec and gbv is not None:
        gbv = (gbv, r(N, 3, H))
    a = ES.adjoint_epi_ln_launch(epi, gbx, gbv, ln)
    b = ES.adjoint_epi_ln_composite(epi, gbx, gbv, ln)
    for i, (ta, tb) in enumerate(zip(a, b)):
        if tb is None:
            continue
        assert ta is not None, i
        assert _rel(ta, tb) < tol, (i, _rel(ta, tb))


@pytest.mark.parametrize("record", [True, False])
@pytest.mark.parametrize("dr", ["1", "0"])
@pytest.mark.parametrize("out_norm", [True, False])
def test_hand_second_order_on_model(monkeypatch, dr, out_norm, record):
    """Training gradients (E + F loss through the create_graph force pass) of the hand second order vs
    autograd over the composite; ``record``: the force pass runs inside second_order_expected() (as
    the training steps do) and hands its record to the second order instead of it being re-run."""
    from torchmdnet import et_stack as ES
    from torchmdnet.models.model import create_model
    monkeypatch.setattr(ES, "DR_MODE", dr)
    args = yaml_args("equivariant-transformer", embedding_dimension=64, num_layers=3, derivative=True,
                     precision=64)
    torch.manual_seed(0)
    model = create_model(args).to(DEV)
    model.representation_model.out_norm.elementwise_affine = True
    if not out_norm:  # fuse_norm needs eps 1e-5: any other eps keeps the norm outside the stack
        model.representation_model.out_norm.eps = 1e-6
    with torch.no_grad():
        model.representation_model.out_norm.weight.add_(0.1 * torch.randn(64, device=DEV, dtype=torch.float64))
    z, pos, batch = O.qm9_like(5, 8)
    z, pos, batch = z.to(DEV), pos.to(DEV), batch.to(DEV)
    torch.manual_seed(1)
    y_t, f_t = torch.randn(5, 1, device=DEV, dtype=torch.float64), torch.randn_like(pos)
    calls = []
    orig = ES._second_order
    monkeypatch.setattr(ES, "_second_order", lambda *a, **k: calls.append(1) or orig(*a, **k))
    grads = []
    for mode in ("hand", "composite"):
        monkeypatch.setattr(ES, "SECOND_ORDER", mode)
        params = [p for p in model.parameters() if p.requires_grad]
        with ES.second_order_expected(record):
            y, neg_dy = model(z, pos.clone(), batch)
        loss = ((y - y_t) ** 2).mean() + ((neg_dy - f_t) ** 2).mean()
        grads.append(torch.autograd.grad(loss, params, allow_unused=True))
    assert calls
    n = 0
    for a, b in zip(*grads):
        if b is None:
            continue
        assert _rel(a, b) < 1e-9
        n += 1
    assert n > 30


@pytest.mark.parametrize("dtype,tol", [(torch.float64, 1e-11), (torch.float32, 2e-5)])
@pytest.mark.parametrize("rbf,cl", [("expnorm", 0.0), ("expnorm", 0.7), ("gauss", 0.0)])
def test_edge_geometry_second_order_hand_matches_composite(monkeypatch, dtype, tol, rbf, cl):
    """tmdnet_edge_geom_bwd2 against autograd's double differentiation of the composite geometry
    (RBF basis, cosine cutoff incl. the shifted form, unit vectors, self edges), every input."""
    import types
    from torchmdnet import _native as nat
    from torchmdnet import kernels as K
    torch.manual_seed(0)
    E, R, cu = 3000, 64, 5.0
    src = torch.randint(0, 100, (E,), device=DEV, dtype=torch.int32)
    dst = torch.randint(0, 100, (E,), device=DEV, dtype=torch.int32)
    dst[:50] = src[:50]
    deltas = torch.randn(E, 3, device=DEV, dtype=dtype) * 2.2
    deltas[src == dst] = 0
    dist = deltas.norm(dim=1)
    if rbf == "expnorm":
        start = torch.exp(torch.scalar_tensor(-cu + cl, dtype=dtype))
        mu = torch.linspace(float(start), 1, R, dtype=dtype, device=DEV)
        beta = torch.full((R,), float((2 / R * (1 - start)) ** -2), dtype=dtype, device=DEV)
        rtype = nat.RBF_EXPNORM
    else:
        mu = torch.linspace(cl, cu, R, dtype=dtype, device=DEV)
        beta = torch.full((R,), -0.5 / float(mu[1] - mu[0]) ** 2, dtype=dtype, device=DEV)
        rtype = nat.RBF_GAUSS
    graph = types.SimpleNamespace(src=src, dst=dst)
    gf0, gC0, gu0 = torch.randn(E, R, device=DEV, dtype=dtype), torch.randn(E, device=DEV, dtype=dtype), \
        torch.randn(E, 3, device=DEV, dtype=dtype)
    c1, c2 = torch.randn(E, 3, device=DEV, dtype=dtype), torch.randn(E, device=DEV, dtype=dtype)
    out = []
    for mode in ("hand", "composite"):
        monkeypatch.setattr(K, "HEAD_SECOND_ORDER", mode)
        leaves = [t.clone().requires_grad_(True) for t in (deltas, dist, gf0, gC0, gu0)]
        g_dl, g_r = K._EdgeGeomBwd.apply(*leaves, graph, mu, beta, cl, cu, rtype)
        loss = (g_dl * c1).sum() + (g_r * c2).sum()
        out.append(torch.autograd.grad(loss, leaves, allow_unused=True))
    for i, (a, b) in enumerate(zip(*out)):
        assert a is not None and b is not None, i
        assert torch.isfinite(a).all(), i
        assert _rel(a, b) < tol, (i, _rel(a, b))


def test_neighbor_embedding_second_order_hand_matches_composite(monkeypatch):
    """tmdnet_nbr_embed_bwd2 (destination pass + source pass over the reversed edges) against autograd's
    double differentiation of the composite, fp64, with non-symmetric cotangents on every output."""
    from torchmdnet import kernels
    torch.manual_seed(4)
    z, pos, batch = O.qm9_like(3)
    g = kernels.build_graph(pos.to(DEV), batch.to(DEV), 0.0, 5.0, 64 * pos.shape[0], loop=True)
    N, H, E = pos.shape[0], 64, g.n_edges
    T = g.transpose.long()
    x0 = torch.randn(N, H, dtype=torch.float64, device=DEV)
    w0 = torch.randn(E, H, dtype=torch.float64, device=DEV)
    w0 = (w0 + w0[T]) / 2
    C0 = torch.rand(E, dtype=torch.float64, device=DEV)
    C0 = (C0 + C0[T]) / 2
    go0 = torch.randn(N, H, dtype=torch.float64, device=DEV)
    wts = [torch.randn(N, H, dtype=torch.float64, device=DEV), torch.randn(E, H, dtype=torch.float64, device=DEV),
           torch.randn(E, dtype=torch.float64, device=DEV)]
    res = []
    for mode in ("hand", "composite"):
        monkeypatch.setattr(kernels, "HEAD_SECOND_ORDER", mode)
        leaves = [t.clone().requires_grad_(True) for t in (go0, x0, w0, C0)]
        a = kernels._NbrEmbedBwd.apply(*leaves, g)
        res.append(torch.autograd.grad(sum((t * u).sum() for t, u in zip(a, wts)), leaves, allow_unused=True))
    for i, (p_, q_) in enumerate(zip(*res)):
        assert p_ is not None and q_ is not None, i
        assert _rel(p_, q_) < 1e-11, (i, _rel(p_, q_))


_TN_WIDE = [(678, 640, 128, True, 678), (2034, 384, 128, False, 2034), (678, 128, 0, True, 678),
            (12548, 128, 64, True, 0), (5000, 96, 64, True, 1200), (37, 100, 36, False, 5),
            (12548, 4096, 64, True, 12548), (3, 4, 8, True, 0)]
# every problem reads <= 32 columns of B: the 32-column tile form (the dk/dv weight gradient's shape)
_TN_NARROW = [(5210, 4096, 32, True, 10420), (5000, 70, 20, True, 900), (678, 128, 0, True, 678),
              (37, 100, 31, False, 5), (12548, 96, 32, False, 0), (3, 4, 8, True, 0)]


@pytest.mark.parametrize("form", ["1", "2", "4", "5"])  # TMDNET_TN_V: 64-tile, pipelined, bf16x3 LDS / register
@pytest.mark.parametrize("shapes", ["wide", "narrow"])
@pytest.mark.parametrize("use_cb", [False, True])
def test_weight_gradient_tn_gemm_16byte_kernel(monkeypatch, use_cb, shapes, form):
    """The 64 x 64-tile, 16-byte-load TN kernel (every row 16-byte aligned): ragged M / N / K, long K
    (split over the rows), two segments with the ones column on one of them, bias-only problems, beta,
    and the bias written to its own vector (Cb) -- against fp64."""
    from torchmdnet import kernels
    monkeypatch.setenv("TMDNET_TN_V", form)
    torch.manual_seed(4)
    shapes = _TN_WIDE if shapes == "wide" else _TN_NARROW
    probs, refs = [], []
    for K, M, Nb, ones, K2 in shapes:
        A, B = torch.randn(K, M, device=DEV), (torch.randn(K, Nb, device=DEV) if Nb else None)
        N = Nb + int(ones)
        C = torch.randn(M, Nb if (use_cb and ones and Nb) else N, device=DEV)
        Cb = torch.randn(M, device=DEV) if (use_cb and ones and Nb) else None
        p = {"A": A, "B": B, "C": C, "ones": ones}
        if Cb is not None:
            p["Cb"] = Cb
        Bx = B.double() if B is not None else torch.zeros((K, 0), dtype=torch.float64, device=DEV)
        if ones:
            Bx = torch.cat((Bx, torch.ones((K, 1), dtype=torch.float64, device=DEV)), 1)
        ref = A.double().t() @ Bx
        if K2 and Nb:
            A2, B2 = torch.randn(K2, M, device=DEV), torch.randn(K2, Nb, device=DEV)
            p.update(A2=A2, B2=B2)
            B2x = B2.double()
            if ones:
                B2x = torch.cat((B2x, torch.zeros((K2, 1), dtype=torch.float64, device=DEV)), 1)
            ref = ref + A2.double().t() @ B2x
        beta = len(probs) % 2 == 1
        if beta:
            p["beta"] = True
            ref = ref + (torch.cat((C, Cb[:, None]), 1) if Cb is not None else C).double()
        probs.append(p)
        refs.append(ref)
    kernels.wgrad_tn(probs)
    for p, ref in zip(probs, refs):
        got = torch.cat((p["C"], p["Cb"][:, None]), 1) if p.get("Cb") is not None else p["C"]
        assert _rel(got, ref) < 2e-5, (tuple(p["A"].shape), _rel(got, ref))


@pytest.mark.parametrize("form", ["1", "2", "5"])
def test_weight_gradient_tn_gemm_device_row_count(monkeypatch, form):
    """tmdnet_gemm_tn_rows_f32_ws: only rows < *rows of each segment are summed (the found pairs of a
    static-capacity edge list), incl. a count of 0, a count inside a split chunk, and one above K."""
    from torchmdnet import kernels
    monkeypatch.setenv("TMDNET_TN_V", form)
    torch.manual_seed(7)
    K, M, Nb = 15872, 4096 if form != "2" else 512, 64 if form != "2" else 32
    A, B = torch.randn(K, M, device=DEV), torch.randn(K, Nb, device=DEV)
    A2, B2 = torch.randn(K, M, device=DEV), torch.randn(K, Nb, device=DEV)
    for count in (12548, 0, 777, K + 100):
        rows = torch.tensor([count], dtype=torch.int32, device=DEV)
        C, Cb = torch.empty(M, Nb, device=DEV), torch.empty(M, device=DEV)
        kernels.wgrad_tn([{"A": A, "B": B, "A2": A2, "B2": B2, "C": C, "Cb": Cb, "ones": True, "rows": rows}])
        c = min(count, K)
        ref = A[:c].double().t() @ B[:c].double() + A2[:c].double().t() @ B2[:c].double()
        refb = A[:c].double().sum(0)
        assert _rel(C, ref) < 2e-5 and _rel(Cb, refb) < 2e-5, (count, _rel(C, ref), _rel(Cb, refb))


def test_weight_gradient_tn_gemm_matches_library():
    """tmdnet_gemm_tn_f32 (grouped C (+)= A^T B + A2^T B2 over rows, ones column = bias) against
    torch fp64 on the shapes the training step uses (node weights over atoms, 3N vec rows, the head's
    narrow factors, column sums) plus ragged sizes and the 16-wave long-K path."""
    from torchmdnet import kernels
    torch.manual_seed(0)
    dev = torch.device(DEV)
    shapes = [(678, 640, 128, True, 678), (2034, 384, 128, False, 2034), (678, 128, 0, True, 0),
              (37, 65, 33, True, 5), (5000, 96, 64, True, 1200), (1356, 2, 65, False, 0), (3, 1, 7, False, 0)]
    probs, refs = [], []
    for K, M, Nb, ones, K2 in shapes:
        A = torch.randn(K, M, device=dev)
        B = torch.randn(K, Nb, device=dev) if Nb else None
        N = Nb + int(ones)
        if N == 0:
            N, Nb, B = 7, 7, torch.randn(K, 7, device=dev)
        C = torch.randn(M, N, device=dev)
        C0 = C.clone()
        p = {"A": A, "B": B, "C": C, "ones": ones}
        Bx = B.double() if B is not None else torch.zeros((K, 0), dtype=torch.float64, device=dev)
        if ones:
            Bx = torch.cat((Bx, torch.ones((K, 1), dtype=torch.float64, device=dev)), 1)
        ref = A.double().t() @ Bx
        if K2:
            A2, B2 = torch.randn(K2, M, device=dev), torch.randn(K2, Nb, device=dev) if Nb else None
            p.update(A2=A2, B2=B2)
            B2x = B2.double() if B2 is not None else torch.zeros((K2, 0), dtype=torch.float64, device=dev)
            if ones:
                B2x = torch.cat((B2x, torch.zeros((K2, 1), dtype=torch.float64, device=dev)), 1)
            ref = ref + A2.double().t() @ B2x
        if len(probs) % 2:
            p["beta"] = True
            ref = ref + C0.double()
        probs.append(p)
        refs.append(ref)
    kernels.wgrad_tn(probs)
    for p, ref in zip(probs, refs):
        assert _rel(p["C"], ref) < 2e-5, (tuple(p["A"].shape), _rel(p["C"], ref))


def test_embedding_backward_one_hot_tn():
    """tmdnet_embedding_bwd_f32 (both tables of one lookup node, one launch) against index_add in
    fp64, incl. accumulate, strided gradient rows and types that never occur."""
    from torchmdnet import kernels
    torch.manual_seed(0)
    z = torch.randint(0, 10, (678,), device=DEV)
    z[:5] = 99
    g1 = torch.randn(678, 128, device=DEV)
    g2 = torch.randn(678, 256, device=DEV)[:, ::2]  # row stride 256
    outs = kernels.embedding_bwd(z, [g1, g2], 100)
    for g, o in zip((g1, g2), outs):
        ref = torch.zeros(100, 128, dtype=torch.float64, device=DEV).index_add_(0, z, g.double())
        assert _rel(o, ref) < 1e-6
    acc = [o.clone() for o in outs]
    kernels.embedding_bwd(z, [g1, g2], 100, out=acc, accumulate=True)
    for a, o in zip(acc, outs):
        assert _rel(a, 2 * o.double()) < 1e-6
    # through the autograd node the model uses
    w1, w2 = (torch.randn(100, 128, device=DEV, requires_grad=True) for _ in range(2))
    x1, x2 = kernels.embedding(z, w1, w2)
    d1, d2 = torch.autograd.grad((x1 * g1).sum() + (x2 * g1).sum(), (w1, w2))
    ref = torch.zeros(100, 128, dtype=torch.float64, device=DEV).index_add_(0, z, g1.double())
    assert _rel(d1, ref) < 1e-6 and _rel(d2, ref) < 1e-6


def test_embedding_forward_one_launch():
    """tmdnet_embedding_fwd_f32 (both tables of the ET lookup node in one launch) bit-exact against
    index_select: strided table rows, int32 indices, a single row and an empty index vector."""
    from torchmdnet import kernels
    torch.manual_seed(1)
    w1 = torch.randn(100, 128, device=DEV)
    w2 = torch.randn(100, 256, device=DEV)[:, :128]  # row stride 256
    for z in (torch.randint(0, 100, (678,), device=DEV), torch.randint(0, 100, (50001,), device=DEV),
              torch.tensor([99], device=DEV), torch.randint(0, 100, (37,), device=DEV, dtype=torch.int32),
              torch.zeros(0, dtype=torch.int64, device=DEV)):
        outs = kernels.embedding_fwd(z, (w1, w2))
        for w, o in zip((w1, w2), outs):
            assert o.shape == (z.shape[0], 128)
            assert torch.equal(o, w.index_select(0, z.long()))
    w3 = torch.randn(5, 12, device=DEV)  # H = 12: three float4 per row
    z = torch.randint(0, 5, (1000,), device=DEV)
    assert torch.equal(kernels.embedding_fwd(z, (w3,))[0], w3[z])


@pytest.mark.parametrize("rows,fin,fout", [(12548, 64, 128), (678, 256, 128), (37, 7, 5)])
def test_linear_tn_first_and_second_order(rows, fin, fout):
    """kernels.linear (TN-GEMM weight / bias gradients, differentiable backward) against F.linear
    in fp64 autograd: first-order gradients and the force-matching style second order (a loss on the
    input gradient, differentiated w.r.t. the weights / bias / input-gradient seed)."""
    import torch.nn.functional as F
    from torchmdnet import kernels
    torch.manual_seed(1)
    x0 = torch.randn(rows, fin, device=DEV)
    w0 = torch.randn(fout, fin, device=DEV) / fin ** 0.5
    b0 = torch.randn(fout, device=DEV)
    gy0 = torch.randn(rows, fout, device=DEV)
    res = []
    for lin, dt in ((kernels.linear, torch.float32), (F.linear, torch.float64)):
        x, w, b = (t.to(dt).clone().requires_grad_(True) for t in (x0, w0, b0))
        y = lin(x, w, b)
        gx, = torch.autograd.grad(y, x, gy0.to(dt) * torch.tanh(y), create_graph=True)
        loss = (y ** 2).sum() + (gx ** 2).sum()
        res.append(torch.autograd.grad(loss, (w, b)))
    for a, r in zip(*res):
        assert _rel(a, r) < 1e-4


def test_node_weight_grads_tn_match_batched_library(monkeypatch):
    """fp32 training gradients of every parameter (E + F loss through the recorded force pass) with the
    node weights' gradients from the grouped TN GEMMs (NODE_WGRAD=tn, biases as separate ones-column
    outputs, adjoint terms as second row segments) against the batched library GEMMs (bmm)."""
    from torchmdnet import et_stack as ES
    from torchmdnet.models.model import create_model
    args = yaml_args("equivariant-transformer", embedding_dimension=64, num_layers=3, derivative=True,
                     precision=32)
    torch.manual_seed(0)
    model = create_model(args).to(DEV)
    z, pos, batch = O.qm9_like(6, 3)
    z, pos, batch = z.to(DEV), pos.float().to(DEV), batch.to(DEV)
    torch.manual_seed(1)
    y_t, f_t = torch.randn(6, 1, device=DEV), torch.randn_like(pos)
    grads = []
    for mode in ("tn", "bmm"):
        monkeypatch.setattr(ES, "NODE_WGRAD", mode)
        params = [p for p in model.parameters() if p.requires_grad]
        with ES.second_order_expected():
            y, neg_dy = model(z, pos.clone(), batch)
        loss = ((y - y_t) ** 2).mean() + ((neg_dy - f_t) ** 2).mean()
        grads.append(torch.autograd.grad(loss, params, allow_unused=True))
    n = 0
    for a, b in zip(*grads):
        if b is None:
            continue
        assert _rel(a, b) < 1e-4
        n += 1
    assert n > 30


@pytest.mark.parametrize("dtype,tol", [(torch.float64, 1e-12), (torch.float32, 1e-5)])
def test_fused_energy_force_loss(dtype, tol):
    """kernels.mse2 (LNNPStep's E + F loss in one launch, backward in one) against the composite
    y_weight * mse_loss + neg_dy_weight * mse_loss: value and both prediction gradients."""
    import torch.nn.functional as F
    from torchmdnet import kernels
    torch.manual_seed(3)
    py, y = torch.randn(32, 1, device=DEV, dtype=dtype), torch.randn(32, 1, device=DEV, dtype=dtype)
    pf, f = torch.randn(678, 3, device=DEV, dtype=dtype), torch.randn(678, 3, device=DEV, dtype=dtype)
    res = []
    for fn in (lambda a, b: kernels.mse2(a, y, b, f, 0.05, 0.95),
               lambda a, b: 0.05 * F.mse_loss(a, y) + 0.95 * F.mse_loss(b, f)):
        a, b = py.clone().requires_grad_(True), pf.clone().requires_grad_(True)
        loss = fn(a, b)
        ga, gb = torch.autograd.grad(3.0 * loss, (a, b))
        res.append((loss.detach(), ga, gb))
    for u, v in zip(*res):
        assert _rel(u, v) < tol
