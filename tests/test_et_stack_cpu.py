"""CPU check of the ET stack's hand-scheduled forward/backward ORCHESTRATION (torchmdnet/et_stack.py).

The four native launches the stack makes (ET message fwd/bwd, epilogue fwd/bwd) are replaced, in
this test only, by composite PyTorch emulations with the kernels' documented buffer semantics
(strided gradient outputs, TMDNET_ACC_* accumulation, vec == NULL).  What is verified is everything
around them: fused/stacked GEMMs, gradient accumulation across layers, layer-norm backward, the
weight-gradient gating and the composite double backward, against plain autograd over the
reference math.  The kernels themselves are checked on the GPU (test_gpu_parity.py).
"""
import math

import os

import pytest
import torch

from torchmdnet import _native as nat
from torchmdnet import et_stack as ES
from torchmdnet import kernels
from torchmdnet.models.torchmd_et import EquivariantMultiHeadAttention

DT = torch.float64


def _to_inter(t, H, heads, planar):
    """planar [x|v1|v2] H-blocks -> reference per-head interleave (columns)."""
    if t is None or not planar:
        return t
    inv = torch.argsort(ES._v_perm(H, heads, t.device))
    return t[:, inv]


def _to_planar(g, H, heads, planar):
    if g is None or not planar:
        return g
    return g[:, ES._v_perm(H, heads, g.device)]


def _expand_rows(pk, pv, pk_rows):
    """Pair-shared projection rows -> per-edge rows (the kernels' pk_rows indirection)."""
    if pk_rows is None:
        return pk, pv
    r = pk_rows.long()
    return (None if pk is None else pk.index_select(0, r)), (None if pv is None else pv.index_select(0, r))


def pair_index_composite(graph):
    """tmdnet_pair_index restated: canonical edges (src >= dst) numbered row by row in CSR order;
    the other direction takes its reverse's number; unused pair slots point at edge 0."""
    E, N = graph.n_edges, graph.n_nodes
    src, dst, tr = graph.src.long(), graph.dst.long(), graph.transpose.long()
    canon = src >= dst
    pid = torch.cumsum(canon.long(), 0) - 1  # CSR order = row by row, in-row order kept
    pair_row = torch.where(canon, pid, pid[tr.clamp(min=0)])
    pair_edge = torch.zeros((E + N) // 2, dtype=torch.long)
    pair_edge[pid[canon]] = torch.nonzero(canon).flatten()
    return pair_row.to(torch.int32), pair_edge.to(torch.int32)


def _fake_pair_index(graph, pair_row, pair_edge):
    r, e = pair_index_composite(graph)
    pair_row.copy_(r)
    pair_edge.copy_(e)


def _fake_fwd(q, k, v, vec, pk, pv, C, u, graph, heads, xo, vo, flags=0, pk_rows=None):
    pk, pv = _expand_rows(pk, pv, pk_rows)
    N, H = q.shape
    planar = bool(flags & nat.ET_V_PLANAR)
    v, pv = _to_inter(v, H, heads, planar), _to_inter(pv, H, heads, planar)
    vec_ = torch.zeros((N, 3, H), dtype=q.dtype) if vec is None else vec
    a, b = kernels.et_message_composite(q, k, v, vec_, pk, pv, C, u, graph.src.long(), graph.dst.long(),
                                        N, heads, flags & 0xFF00)
    xo.copy_(a)
    vo.copy_(b)


def _fake_bwd(q, k, v, vec, pk, pv, C, u, graph, heads, gx, gvec, gq, gk, gv, gw, gpk, gpv, gC, gu,
              accumulate=0, pk_rows=None, dpk=None, dpv=None, g_r=None):
    pk, pv = _expand_rows(pk, pv, pk_rows)
    dpk, dpv = _expand_rows(dpk, dpv, pk_rows)
    N, H = q.shape
    planar = bool(accumulate & nat.ET_V_PLANAR)
    v, pv = _to_inter(v, H, heads, planar), _to_inter(pv, H, heads, planar)
    with torch.enable_grad():
        ins = [None if t is None else t.detach().clone().requires_grad_(True)
               for t in (q, k, v, vec, pk, pv, C, u)]
        vec_ = torch.zeros((N, 3, H), dtype=q.dtype) if vec is None else ins[3]
        xo, vo = kernels.et_message_composite(ins[0], ins[1], ins[2], vec_, ins[4], ins[5], ins[6], ins[7],
                                              graph.src.long(), graph.dst.long(), N, heads, accumulate & 0xFF00)
        live = [t for t in ins if t is not None]
        g = torch.autograd.grad((xo, vo), live, (gx, gvec), allow_unused=True)
    it = iter(g)
    g = [next(it) if t is not None else None for t in ins]
    z = lambda t, ref: torch.zeros_like(ref) if t is None else t  # noqa: E731
    ag = bool(accumulate & nat.ACC_GRADS)
    put = (lambda d, val: d.add_(val)) if ag else (lambda d, val: d.copy_(val))  # noqa: E731
    put(gq, z(g[0], q))
    put(gk, z(g[1], k))
    put(gv, _to_planar(z(g[2], v), H, heads, planar))
    if gw is not None:
        put(gw, z(g[3], gw) + (gvec if accumulate & nat.ACC_VEC_RESIDUAL else 0))
    if gpk is not None:
        put(gpk, z(g[4], pk))
    if gpv is not None:
        put(gpv, _to_planar(z(g[5], pv), H, heads, planar))
    if g_r is not None:  # dr mode: <g_pk, dpk> + <g_pv, dpv> per edge (dpv in the kernel's row layout);
        # gpk / gpv given as well: the recorded force pass keeps the projection gradient (stored above)
        if not accumulate & nat.ACC_EDGE:
            g_r.zero_()
        if dpk is not None:
            g_r.add_((z(g[4], pk) * dpk).sum(1))
        if dpv is not None:
            g_r.add_((_to_planar(z(g[5], pv), H, heads, planar) * dpv).sum(1))
    if accumulate & nat.ACC_EDGE:
        gC.add_(g[6])
        gu.add_(g[7])
    else:
        gC.copy_(g[6])
        gu.copy_(g[7])


def _fake_epi_fwd(x, vec, vecp, o, veca):
    H = x.shape[1]
    o1, o2, o3 = o[:, :H], o[:, H:2 * H], o[:, 2 * H:]
    if vecp is None:
        return x + o3, veca.clone()
    v1, v2, v3 = vecp[..., :H], vecp[..., H:2 * H], vecp[..., 2 * H:]
    return x + (v1 * v2).sum(1) * o2 + o3, vec + v3 * o1.unsqueeze(1) + veca


def _fake_epi_bwd(gx, gvec, vecp, o, g_vecp, g_o, acc=False):
    if acc:  # accumulate: run into scratch and add
        tv = None if g_vecp is None else torch.zeros_like(g_vecp)
        to = torch.zeros_like(g_o)
        _fake_epi_bwd(gx, gvec, vecp, o, tv, to)
        g_o.add_(to)
        if vecp is not None:
            g_vecp.add_(tv)
        return
    H = gx.shape[1]
    o1, o2 = o[:, :H], o[:, H:2 * H]
    if vecp is None:
        g_o.zero_()
        g_o[:, 2 * H:] = gx
        return
    v1, v2, v3 = vecp[..., :H], vecp[..., H:2 * H], vecp[..., 2 * H:]
    g_o[:, :H] = (gvec * v3).sum(1)
    g_o[:, H:2 * H] = gx * (v1 * v2).sum(1)
    g_o[:, 2 * H:] = gx
    gd = (gx * o2).unsqueeze(1)
    g_vecp[..., :H] = gd * v2
    g_vecp[..., H:2 * H] = gd * v1
    g_vecp[..., 2 * H:] = gvec * o1.unsqueeze(1)


def _fake_epi_ln(x, vec, vecp, o, veca, ln_w, ln_b, xn_out=None, vo_out=None):
    """tmdnet_et_epilogue_ln_fwd restated: epilogue (if o) then the next layer's LayerNorm."""
    xo = vo = None
    if o is not None:
        xo, vo = _fake_epi_fwd(x, vec, vecp, o, veca)
        x = xo
        if vo_out is not None:
            vo = vo_out.copy_(vo)
    xn, mean, rstd = torch.native_layer_norm(x, [x.shape[1]], ln_w, ln_b, ES._EPS)
    if xn_out is not None:
        xn = xn_out.copy_(xn)
    return xo, vo, xn, mean, rstd


def _fake_ln_bwd_epi(g_xn, x, mean, rstd, ln_w, g_res, g_vec, vecp, o, g_vecp, g_o, wrows=None, g_res2=None,
                     acc=False):
    """tmdnet_ln_bwd_epilogue_w restated: residual + LayerNorm backward, then the previous epilogue
    (and the LayerNorm weight gradient's row terms)."""
    g_x, _, _ = torch.ops.aten.native_layer_norm_backward(g_xn, x, [x.shape[1]], mean, rstd, ln_w, None,
                                                          [True, False, False])
    if wrows is not None:
        wrows.copy_(g_xn * (x - mean) * rstd)
    if g_res is not None:
        g_x = g_x + g_res
    if g_res2 is not None:
        g_x = g_x + g_res2
    if o is not None:
        _fake_epi_bwd(g_x, g_vec, vecp, o, g_vecp, g_o, acc=acc)
    return g_x


def _fake_rbf_deriv(r, mu, beta, cl, cu, rbf_type, rows, out):
    rr = r if rows is None else r.index_select(0, rows.long())
    cols = []
    for k in range(mu.shape[0]):  # f_k(r_e) depends on r_e only: d/dr of the column sum
        with torch.enable_grad():
            x = rr.detach().clone().requires_grad_(True)
            fk = kernels.rbf_composite(x, mu, beta, cl, cu, rbf_type)[:, k]
            (g,) = torch.autograd.grad(fk.sum(), x)
        cols.append(g)
    out.copy_(torch.stack(cols, 1))


def _fake_bwd2(ctx, ggs):
    return kernels._ETMessageBwd.composite_backward(ctx, *ggs)


def _fake_bwd2_launch(q, k, v, vec, pk, pv, C, u, graph, heads, gx, gvec, ggs, flags=0, out=None, pk_rows=None,
                      gg_pkv_scale=None):
    """tmdnet_et_message_bwd2_ex restated: the VJP of the message backward by double autograd (``out``
    buffers filled / accumulated as the launch wrapper does; ``pk_rows``: pair-shared projection rows;
    ``gg_pkv_scale``: the projection cotangents are pair rows scaled per edge)."""
    if gg_pkv_scale is not None:
        idx = pk_rows.long()
        sc = gg_pkv_scale.unsqueeze(1)
        ggs = tuple(ggs[:4]) + tuple(None if t is None else t.index_select(0, idx) * sc for t in ggs[4:6]) + tuple(ggs[6:])
    if pk_rows is not None:
        idx = pk_rows.long()
        pk = pk.index_select(0, idx) if pk is not None else None
        pv = pv.index_select(0, idx) if pv is not None else None
    res = _fake_bwd2_core(q, k, v, vec, pk, pv, C, u, graph, heads, gx, gvec, ggs, flags & 0xFF00)
    if not out:
        return res
    d_gx, d_gvec, d_q, d_k, d_v, d_vec, d_pk, d_pv, d_C, d_u = res
    if "gx" in out:
        d_gx = out["gx"].copy_(d_gx)
    if "qkv" in out:
        out["qkv"].copy_(torch.cat((d_q, d_k, d_v), 1))
    if "pkv" in out:
        out["pkv"].copy_(torch.cat([t for t in (d_pk, d_pv) if t is not None], 1))
    if "C" in out:
        if out.get("edge_overwrite"):
            out["C"].copy_(d_C)
            out["u"].copy_(d_u)
        else:
            out["C"].add_(d_C)
            out["u"].add_(d_u)
        d_C, d_u = out["C"], out["u"]
    if "gvec" in out:
        out["gvec"].add_(d_gvec)
        d_gvec = out["gvec"]
    return d_gx, d_gvec, d_q, d_k, d_v, d_vec, d_pk, d_pv, d_C, d_u


def _fake_bwd2_core(q, k, v, vec, pk, pv, C, u, graph, heads, gx, gvec, ggs, acts=0):
    N, H = q.shape
    vec_ = torch.zeros((N, 3, H), dtype=q.dtype) if vec is None else vec
    with torch.enable_grad():
        prim = [None if t is None else t.detach().clone().requires_grad_(True)
                for t in (q, k, v, vec_, pk, pv, C, u)]
        seeds = [gx.detach().clone().requires_grad_(True), gvec.detach().clone().requires_grad_(True)]
        xo, vo = kernels.et_message_composite(*prim, graph.src.long(), graph.dst.long(), N, heads, acts)
        live = [t for t in prim if t is not None]
        first = torch.autograd.grad((xo, vo), live, seeds, create_graph=True, allow_unused=True)
        it = iter(first)
        first = [next(it) if t is not None else None for t in prim]
        sel = [(f_, g_) for f_, g_ in zip(first, ggs) if f_ is not None and g_ is not None and g_.numel()]
        ins = seeds + live
        second = torch.autograd.grad([a for a, _ in sel], ins, [b for _, b in sel], allow_unused=True)
    z = lambda t, ref: torch.zeros_like(ref) if t is None else t  # noqa: E731
    it = iter(second[2:])
    d = [next(it) if t is not None else None for t in prim]
    return (z(second[0], gx), z(second[1], gvec), z(d[0], q), z(d[1], k), z(d[2], v),
            None if vec is None else z(d[3], vec_), None if pk is None else z(d[4], pk),
            None if pv is None else z(d[5], pv), z(d[6], C), z(d[7], u))


@pytest.fixture
def emulated(monkeypatch):
    monkeypatch.setattr(kernels, "et_message_fwd_launch", _fake_fwd)
    monkeypatch.setattr(kernels, "pair_index_launch", _fake_pair_index)
    monkeypatch.setattr(kernels, "et_message_bwd_launch", _fake_bwd)
    monkeypatch.setattr(kernels, "et_message_bwd2", _fake_bwd2)
    monkeypatch.setattr(kernels, "et_message_bwd2_launch", _fake_bwd2_launch)
    monkeypatch.setattr(ES, "adjoint_epi_ln_launch", ES.adjoint_epi_ln_composite)
    monkeypatch.setattr(kernels, "rbf_deriv_launch", _fake_rbf_deriv)
    monkeypatch.setattr(ES, "_epilogue_fwd", _fake_epi_fwd)
    monkeypatch.setattr(ES, "_epilogue_bwd", _fake_epi_bwd)
    monkeypatch.setattr(ES, "_epi_ln", _fake_epi_ln)
    monkeypatch.setattr(ES, "_ln_bwd_epi", _fake_ln_bwd_epi)


def _system(n_mol=3, seed=0, cutoff=4.0):
    g = torch.Generator().manual_seed(seed)
    sizes = [5, 7, 4][:n_mol]
    pos = torch.cat([torch.randn(s, 3, generator=g, dtype=DT) * 1.3 for s in sizes])
    batch = torch.cat([torch.full((s,), i, dtype=torch.long) for i, s in enumerate(sizes)])
    d = (pos[:, None] - pos[None]).norm(dim=-1)
    adj = (d < cutoff) & (batch[:, None] == batch[None])
    ei = adj.nonzero().t().contiguous()  # includes self loops (loop=True)
    graph, perm = kernels.EdgeGraph.from_edge_index(ei, pos.shape[0])
    ei = ei[:, perm]
    vecs = pos[ei[0]] - pos[ei[1]]
    r = vecs.norm(dim=-1)
    return pos.shape[0], graph, r, vecs


def _inputs(n, graph, r, vecs, H, R, seed=1):
    g = torch.Generator().manual_seed(seed)
    mu = torch.linspace(0, 4, R, dtype=DT)
    f = torch.exp(-((r[:, None] - mu) ** 2))  # symmetric per-edge features
    C = 0.5 * (torch.cos(r * math.pi / 4.0) + 1.0)
    u = torch.where((r > 0)[:, None], vecs / torch.where(r > 0, r, torch.ones_like(r))[:, None], vecs)
    x = torch.randn(n, H, generator=g, dtype=DT)
    return x, f, C, u


def _layers(n_layers, H, R, heads, infl, seed=2):
    torch.manual_seed(seed)
    layers = torch.nn.ModuleList([
        EquivariantMultiHeadAttention(H, R, infl, heads, torch.nn.SiLU, "silu", 0.0, 4.0, DT)
        for _ in range(n_layers)])
    with torch.no_grad():  # non-trivial biases / norms
        for p in layers.parameters():
            p.add_(0.1 * torch.randn_like(p))
    return layers


def _meta_for(layers, graph):
    l0 = layers[0]
    return ES._Meta(graph, l0.num_heads, l0.hidden_channels, l0.dk_proj is not None, l0.dv_proj is not None,
                    len(layers), None, None)


@pytest.mark.parametrize("planar", [False, True])
@pytest.mark.parametrize("batched", [True, False])
@pytest.mark.parametrize("infl", ["both", "keys", "values", "none"])
def test_stack_forward_and_grads_match_composite(emulated, monkeypatch, infl, batched, planar):
    if not batched:  # per-layer dk/dv GEMMs (the large-system path)
        monkeypatch.setattr(ES, "BATCH_DKV_BYTES", 0)
    if planar:  # planar v / dv rows (permuted weight rows; the large-system path)
        monkeypatch.setattr(ES, "PLANAR_MIN_EDGES", 0)
    H, R, heads = 16, 8, 4
    n, graph, r, vecs = _system()
    x, f, C, u = _inputs(n, graph, r, vecs, H, R)
    layers = _layers(3, H, R, heads, infl)
    params = [p for l in layers for p in ES.layer_params(l)]
    leaves = [t.clone().requires_grad_(True) for t in (x, f, C, u)]
    xo, vo = ES.et_stack(layers, leaves[0], graph, leaves[1], leaves[2], leaves[3])
    meta = _meta_for(layers, graph)
    ref_leaves = [t.clone().requires_grad_(True) for t in (x, f, C, u)]
    xr, vr = ES.composite_stack(meta, *ref_leaves, params)
    assert torch.allclose(xo, xr, atol=1e-12) and torch.allclose(vo, vr, atol=1e-12)
    gx, gv = torch.randn_like(xo), torch.randn_like(vo)
    wrt = leaves if infl != "none" else [leaves[0], leaves[2], leaves[3]]
    rwrt = ref_leaves if infl != "none" else [ref_leaves[0], ref_leaves[2], ref_leaves[3]]
    a = torch.autograd.grad((xo, vo), wrt + params, (gx, gv), allow_unused=True)
    b = torch.autograd.grad((xr, vr), rwrt + params, (gx, gv), allow_unused=True)
    for i, (ga, gb) in enumerate(zip(a, b)):
        if gb is None:
            assert ga is None or torch.count_nonzero(ga) == 0, i
            continue
        assert torch.allclose(ga, gb, atol=1e-11, rtol=1e-9), i


def test_stack_stacked_parameters_alias_and_survive_updates(emulated):
    H, R, heads = 16, 8, 4
    n, graph, r, vecs = _system()
    x, f, C, u = _inputs(n, graph, r, vecs, H, R)
    layers = _layers(2, H, R, heads, "both")
    ES.et_stack(layers, x, graph, f, C, u)
    lw = layers[0]._stacked
    qkv = lw.bufs["qkv_w"]
    assert layers[0].k_proj.weight.data_ptr() == qkv.data_ptr() + H * H * qkv.element_size()
    dkv = layers._tmd_stack.bufs["w"]  # all layers' [dk; dv] rows: layer 1's dk after layer 0's 4H rows
    assert layers[1].dk_proj.weight.data_ptr() == dkv.data_ptr() + 4 * H * R * dkv.element_size()
    with torch.no_grad():  # optimiser-style in-place update shows through the stacked buffer
        layers[0].k_proj.weight.add_(1.0)
    assert torch.equal(qkv[H:2 * H], layers[0].k_proj.weight)
    sd = {k: v.clone() for k, v in layers.state_dict().items()}
    layers.load_state_dict(sd)
    assert lw.bufs["qkv_w"] is qkv  # in-place load keeps the aliasing


@pytest.mark.parametrize("batched", [True, False])
def test_stack_force_pass_skips_weight_grads_but_training_gets_them(emulated, monkeypatch, batched):
    """autograd.grad wrt inputs: weight gradients not requested -> not computed; loss.backward
    through a create_graph force pass -> weight gradients equal the composite reference (the second
    order re-runs the layers with the message Functions)."""
    H, R, heads = 16, 8, 4
    n, graph, r, vecs = _system()
    x, f, C, u = _inputs(n, graph, r, vecs, H, R)
    if not batched:
        monkeypatch.setattr(ES, "BATCH_DKV_BYTES", 0)
    layers = _layers(2, H, R, heads, "both")
    params = [p for l in layers for p in ES.layer_params(l)]
    calls = []
    orig = ES._backward_layers

    def spy(meta, gX, gV, f_, C_, u_, params_, acts, need_ws, **kw):
        calls.append(tuple(need_ws))
        return orig(meta, gX, gV, f_, C_, u_, params_, acts, need_ws, **kw)

    ES._backward_layers = spy
    try:
        outs = []
        for fused in (True, False):
            leaves = [t.clone().requires_grad_(True) for t in (x, f, C, u)]
            if fused:
                xo, vo = ES.et_stack(layers, leaves[0], graph, leaves[1], leaves[2], leaves[3])
            else:
                xo, vo = ES.composite_stack(_meta_for(layers, graph), *leaves, params)
            e = (xo ** 2).sum() + (vo ** 2).sum()
            g = torch.autograd.grad(e, leaves, create_graph=True)
            loss = e + sum((gi ** 2).sum() for gi in g)
            for p in params:
                p.grad = None
            loss.backward()
            outs.append([p.grad.clone() for p in params])
    finally:
        ES._backward_layers = orig
    assert calls[0] == (False, False)  # the force pass
    assert (True, True) in calls[1:]   # loss.backward (the second order's passes run too)
    for a, b in zip(*outs):
        assert torch.allclose(a, b, atol=1e-10, rtol=1e-8)


def test_stack_partial_parameter_request(emulated):
    H, R, heads = 16, 8, 4
    n, graph, r, vecs = _system()
    x, f, C, u = _inputs(n, graph, r, vecs, H, R)
    layers = _layers(2, H, R, heads, "both")
    xo, vo = ES.et_stack(layers, x, graph, f, C, u)
    (g,) = torch.autograd.grad(xo.sum() + vo.sum(), [layers[1].o_proj.weight])
    xr, vr = ES.composite_stack(_meta_for(layers, graph), x, f, C, u,
                                [p for l in layers for p in ES.layer_params(l)])
    (gr,) = torch.autograd.grad(xr.sum() + vr.sum(), [layers[1].o_proj.weight])
    assert torch.allclose(g, gr, atol=1e-11)


# a pairwise covering array of (record, infl, batched, planar, rbf_type): every pair of values of any two
# switches occurs in some case (6 cases instead of the 48 of the full grid, ~30 s of CPU each;
# TMDNET_FULL_GRID=1 runs all 48)
_DR_GRID = ([(r, i, b, p, t) for r in (True, False) for i in ("both", "keys", "values") for b in (True, False)
             for p in (False, True) for t in (nat.RBF_GAUSS, nat.RBF_EXPNORM)]
            if os.environ.get("TMDNET_FULL_GRID") == "1" else
            [(True, "both", True, False, nat.RBF_GAUSS), (False, "both", False, True, nat.RBF_EXPNORM),
             (True, "keys", False, True, nat.RBF_GAUSS), (False, "keys", True, False, nat.RBF_EXPNORM),
             (True, "values", True, True, nat.RBF_EXPNORM), (False, "values", False, False, nat.RBF_GAUSS)])


@pytest.mark.parametrize("record,infl,batched,planar,rbf_type", _DR_GRID)
def test_stack_dr_mode_force_pass_and_second_order(emulated, monkeypatch, record, infl, batched, planar, rbf_type):
    """Force pass with f = rbf(r) declared (the ET model's fixed basis): the stack returns the edge
    gradient on r directly (dr mode, no projection gradient); forces and the force-matching second
    order (weight gradients through a create_graph force pass) equal plain autograd.  ``record``: the
    create_graph force pass runs in dr mode keeping the projection gradient and hands its record (with
    the pair rows' d(dk,dv)/dr, which the second order scales per edge instead of forming gb_f W^T) to
    the hand second order (RECORD_IN_FORCE_PASS) instead of the second order re-running it."""
    monkeypatch.setattr(ES, "DR_MODE", "1")  # also on the stacked (batched) projection path
    monkeypatch.setattr(ES, "RECORD_IN_FORCE_PASS", record)
    if not batched:
        monkeypatch.setattr(ES, "BATCH_DKV_BYTES", 0)
    if planar:
        monkeypatch.setattr(ES, "PLANAR_MIN_EDGES", 0)
    H, R, heads = 16, 8, 4
    cl, cu = 0.0, 4.0
    n, graph, r, vecs = _system()
    x, _, C, u = _inputs(n, graph, r, vecs, H, R)
    if rbf_type == nat.RBF_GAUSS:
        mu, beta = torch.linspace(0, 4, R, dtype=DT), torch.full((R,), -1.0, dtype=DT)
    else:
        mu, beta = torch.linspace(math.exp(-4.0), 1.0, R, dtype=DT), torch.full((R,), 3.0, dtype=DT)
    layers = _layers(2, H, R, heads, infl)
    params = [p for l in layers for p in ES.layer_params(l)]
    modes = []
    orig = ES._backward_layers

    def spy(*a, **kw):
        modes.append((kw.get("dr", False), kw.get("record") is not None))
        return orig(*a, **kw)

    monkeypatch.setattr(ES, "_backward_layers", spy)
    outs = []
    for fused in (True, False):
        rl, xl, Cl, ul = (t.clone().requires_grad_(True) for t in (r, x, C, u))
        f = kernels.rbf_composite(rl, mu, beta, cl, cu, rbf_type)
        if fused:
            xo, vo = ES.et_stack(layers, xl, graph, f, Cl, ul, rbf=(rl, mu, beta, cl, cu, rbf_type))
        else:
            xo, vo = ES.composite_stack(_meta_for(layers, graph), xl, f, Cl, ul, params)
        e = (xo ** 2).sum() + 0.3 * (vo ** 2).sum()
        with ES.second_order_expected():
            g = torch.autograd.grad(e, [rl, xl, Cl, ul], create_graph=True)
        loss = e + sum((gi ** 2).sum() for gi in g)
        for p in params:
            p.grad = None
        loss.backward()
        outs.append([t.detach().clone() for t in g] + [p.grad.clone() for p in params])
    hand = not planar  # the hand second order covers the reference row layout
    if record and hand:  # force pass recorded (dr mode + kept projection gradient), no re-run later
        assert modes[0] == (True, True) and not any(rec for _, rec in modes[1:])
    else:  # force pass in dr mode; loss.backward's passes not
        assert modes[0] == (True, False) and not modes[1][0]
    for i, (a, b) in enumerate(zip(*outs)):
        assert torch.allclose(a, b, atol=1e-10, rtol=1e-8), i


@pytest.mark.parametrize("batched", [True, False])
def test_stack_fused_out_norm(emulated, monkeypatch, batched):
    """The model's out_norm fused into the last epilogue (et_stack(out_norm=...)): outputs, the force
    pass (LayerNorm + epilogue backward in one kernel, dr mode), and training gradients of every
    parameter including the norm's (loss.backward through a create_graph force pass)."""
    if not batched:
        monkeypatch.setattr(ES, "BATCH_DKV_BYTES", 0)
    H, R, heads = 16, 8, 4
    n, graph, r, vecs = _system()
    x, _, C, u = _inputs(n, graph, r, vecs, H, R)
    mu, beta = torch.linspace(0, 4, R, dtype=DT), torch.full((R,), -1.0, dtype=DT)
    layers = _layers(2, H, R, heads, "both")
    norm = torch.nn.LayerNorm(H, dtype=DT)
    with torch.no_grad():
        norm.weight.add_(0.2 * torch.randn(H, dtype=DT))
        norm.bias.add_(0.1 * torch.randn(H, dtype=DT))
    params = [p for l in layers for p in ES.layer_params(l)] + [norm.weight, norm.bias]
    outs = []
    for fused in (True, False):
        rl, xl, Cl, ul = (t.clone().requires_grad_(True) for t in (r, x, C, u))
        f = kernels.rbf_composite(rl, mu, beta, 0.0, 4.0, nat.RBF_GAUSS)
        if fused:
            xo, vo = ES.et_stack(layers, xl, graph, f, Cl, ul, rbf=(rl, mu, beta, 0.0, 4.0, nat.RBF_GAUSS),
                                 out_norm=norm)
        else:
            xo, vo = ES.composite_stack(_meta_for(layers, graph), xl, f, Cl, ul, params[:-2])
            xo = norm(xo)
        e = (xo ** 3).sum() + 0.3 * (vo ** 2).sum()
        g = torch.autograd.grad(e, [rl, xl, Cl, ul], create_graph=True)
        loss = e + sum((gi ** 2).sum() for gi in g)
        for p in params:
            p.grad = None
        loss.backward()
        outs.append([xo.detach().clone(), vo.detach().clone()] + [t.detach().clone() for t in g] +
                    [p.grad.clone() for p in params])
    for i, (a, b) in enumerate(zip(*outs)):
        assert torch.allclose(a, b, atol=1e-10, rtol=1e-8), i


# every distance_influence mode against both values of each switch (pairwise cover of the 32-case grid:
# each case takes ~20 s of emulated double backward on the CPU); TMDNET_FULL_GRID=1 runs all 32
_SO_GRID = ([(i, b, d, o) for i in ("both", "keys", "values", "none") for b in (True, False) for d in ("1", "0")
             for o in (False, True)] if os.environ.get("TMDNET_FULL_GRID") == "1" else
            [("both", True, "1", True), ("both", False, "0", False), ("keys", True, "0", False),
             ("keys", False, "1", True), ("values", True, "1", False), ("values", False, "0", True),
             ("none", True, "0", True), ("none", False, "1", False)])


@pytest.mark.parametrize("infl,batched,dr,out_norm", _SO_GRID)
def test_hand_second_order_matches_composite(emulated, monkeypatch, infl, batched, dr, out_norm):
    """The hand-scheduled second order (et_stack._second_order: recorded first-order pass, its adjoint
    in forward layer order, a backward with injected cotangents) against autograd's double
    differentiation of the recomputed stack: weight gradients AND the gradients of every stack input
    (x, r, C, u and the force seeds, through a loss on the force-pass outputs)."""
    monkeypatch.setattr(ES, "DR_MODE", dr)
    if not batched:
        monkeypatch.setattr(ES, "BATCH_DKV_BYTES", 0)
    H, R, heads = 16, 8, 4
    n, graph, r, vecs = _system()
    x, _, C, u = _inputs(n, graph, r, vecs, H, R)
    mu, beta = torch.linspace(math.exp(-4.0), 1.0, R, dtype=DT), torch.full((R,), 3.0, dtype=DT)
    layers = _layers(3, H, R, heads, infl)
    norm = torch.nn.LayerNorm(H, dtype=DT) if out_norm else None
    if norm is not None:
        with torch.no_grad():
            norm.weight.add_(0.2 * torch.randn(H, dtype=DT))
    params = [p for l in layers for p in ES.layer_params(l)] + ([norm.weight, norm.bias] if norm else [])
    calls = []
    orig = ES._second_order

    def spy(*a, **kw):
        calls.append(1)
        return orig(*a, **kw)

    monkeypatch.setattr(ES, "_second_order", spy)
    outs = []
    for mode in ("hand", "composite"):
        monkeypatch.setattr(ES, "SECOND_ORDER", mode)
        rl, xl, Cl, ul = (t.clone().requires_grad_(True) for t in (r, x, C, u))
        f = kernels.rbf_composite(rl, mu, beta, 0.0, 4.0, nat.RBF_EXPNORM)
        xo, vo = ES.et_stack(layers, xl, graph, f, Cl, ul, rbf=(rl, mu, beta, 0.0, 4.0, nat.RBF_EXPNORM),
                             out_norm=norm)
        # a head-like readout that keeps the force seeds gX / gV data-dependent
        e = (torch.tanh(xo) ** 2).sum() + 0.3 * ((vo ** 2).sum(1) * xo).sum()
        g = torch.autograd.grad(e, [rl, xl, Cl, ul], create_graph=True, allow_unused=True)
        loss = e + sum((gi * torch.randn(gi.shape, dtype=DT, generator=torch.Generator().manual_seed(9))).sum() ** 2
                       for gi in g if gi is not None)
        grads = torch.autograd.grad(loss, params + [rl, xl, Cl, ul], allow_unused=True)
        outs.append([None if t is None else t.detach() for t in grads])
    assert calls, "the hand-scheduled second order did not run"
    for i, (a, b) in enumerate(zip(*outs)):
        if b is None:
            assert a is None or torch.count_nonzero(a) == 0, i
            continue
        assert a is not None, i
        assert torch.allclose(a, b, atol=1e-10, rtol=1e-8), (i, (a - b).abs().max())


def _ref_stack(layers, x, f, C, u, src, dst, act_kv, act_at):
    """Independent restatement of the reference layer loop (torchmd_et.py:177-184, 293-347) with the
    activations given as plain functions."""
    N, H = x.shape
    vec = torch.zeros((N, 3, H), dtype=x.dtype)
    for layer in layers:
        heads, d = layer.num_heads, H // layer.num_heads
        xn = torch.nn.functional.layer_norm(x, (H,), layer.layernorm.weight, layer.layernorm.bias, 1e-5)
        q = layer.q_proj(xn).view(N, heads, d)
        k = layer.k_proj(xn).view(N, heads, d)
        v = layer.v_proj(xn).view(N, heads, 3 * d)
        vec1, vec2, vec3 = torch.split(layer.vec_proj(vec), H, dim=-1)
        att = q[dst] * k[src]
        if layer.dk_proj is not None:
            att = att * act_kv(layer.dk_proj(f)).view(-1, heads, d)
        att = act_at(att.sum(-1)) * C.unsqueeze(1)
        vj = v[src]
        if layer.dv_proj is not None:
            vj = vj * act_kv(layer.dv_proj(f)).view(-1, heads, 3 * d)
        xm, v1, v2 = torch.split(vj, d, dim=2)
        xm = xm * att.unsqueeze(2)
        vm = vec.view(N, 3, heads, d)[src] * v1.unsqueeze(1) + v2.unsqueeze(1) * u.view(-1, 3, 1, 1)
        xa = torch.zeros(N, heads, d, dtype=x.dtype).index_add(0, dst, xm).view(N, H)
        va = torch.zeros(N, 3, heads, d, dtype=x.dtype).index_add(0, dst, vm).view(N, 3, H)
        o1, o2, o3 = torch.split(layer.o_proj(xa), H, dim=1)
        x = x + (vec1 * vec2).sum(dim=1) * o2 + o3
        vec = vec + vec3 * o1.unsqueeze(1) + va
    return x, vec


@pytest.mark.parametrize("acts", [("tanh", "ssp"), ("sigmoid", "tanh"), ("ssp", "sigmoid")])
def test_stack_activations_match_reference_loop(emulated, acts):
    """Non-SiLU `activation` / `attn_activation` (reference act_class_mapping, utils.py:579-584): the
    stack's launches carry the activation codes (TMDNET_ET_ACT flags) through the forward, the
    first-order backward and the second order, against a plain restatement of the layer loop."""
    from torchmdnet.models.utils import act_class_mapping
    H, R, heads = 16, 8, 4
    n, graph, r, vecs = _system()
    x, f, C, u = _inputs(n, graph, r, vecs, H, R)
    torch.manual_seed(2)
    layers = torch.nn.ModuleList([
        EquivariantMultiHeadAttention(H, R, "both", heads, act_class_mapping[acts[0]], acts[1], 0.0, 4.0, DT)
        for _ in range(2)])
    with torch.no_grad():
        for p in layers.parameters():
            p.add_(0.1 * torch.randn_like(p))
    fns = {"tanh": torch.tanh, "sigmoid": torch.sigmoid,
           "ssp": lambda t: torch.nn.functional.softplus(t) - 0.693147182464599609375}
    src, dst = graph.src.long(), graph.dst.long()
    leaves = [t.clone().requires_grad_(True) for t in (x, f, C, u)]
    xo, vo = ES.et_stack(layers, leaves[0], graph, leaves[1], leaves[2], leaves[3])
    ref_leaves = [t.clone().requires_grad_(True) for t in (x, f, C, u)]
    xr, vr = _ref_stack(layers, *ref_leaves, src, dst, fns[acts[0]], fns[acts[1]])
    assert torch.allclose(xo, xr, atol=1e-12) and torch.allclose(vo, vr, atol=1e-12)
    params = list(layers.parameters())
    gx, gv = torch.randn_like(xo), torch.randn_like(vo)
    a = torch.autograd.grad((xo, vo), leaves + params, (gx, gv), create_graph=True)
    b = torch.autograd.grad((xr, vr), ref_leaves + params, (gx, gv), create_graph=True)
    for ga, gb in zip(a, b):
        assert torch.allclose(ga, gb, atol=1e-11, rtol=1e-9)
    # second order: a scalar of the first-order input gradients, differentiated w.r.t. the parameters
    sa = sum((t * t).sum() for t in a[:4])
    sb = sum((t * t).sum() for t in b[:4])
    for ga, gb in zip(torch.autograd.grad(sa, params), torch.autograd.grad(sb, params)):
        assert torch.allclose(ga, gb, atol=1e-10, rtol=1e-8)
