"""GPU checks of the ET forward's node-fused mixes (csrc/et_nodemix.hip; reference torchmd_et.py:181-184,
262-312): ``tmdnet_et_ln_mix_f32`` (LayerNorm + [q|k|v] + vec_proj in one launch) and
``tmdnet_et_oproj_epilogue_f32`` (o_proj + the layer epilogue) against the three-launch form they replace
and a PyTorch fp32 restatement, then the C2 model end to end with the fusion on and off (energies,
forces, force-loss parameter gradients) and against the fp64 oracle."""
import pytest
import torch

from conftest import yaml_args

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return float((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30))


def _inputs(N, H, first, seed=0):
    g = torch.Generator().manual_seed(seed)
    r = lambda *s: torch.randn(*s, generator=g).to(DEV)  # noqa: E731
    xa, x, veca = r(N, H), r(N, H), r(N, 3, H)
    vec = None if first else r(N, 3, H)
    vecp = None if first else r(N, 3, 3 * H)
    o_w, o_b = r(3 * H, H) / H ** 0.5, r(3 * H)
    return xa, x, vec, vecp, veca, o_w, o_b


@pytest.mark.parametrize("N,H,first", [(678, 128, False), (678, 128, True), (37, 64, False), (100, 256, False),
                                       (1, 128, False)])
def test_oproj_epilogue_matches_two_launch_form(N, H, first):
    from torchmdnet import et_stack, kernels
    xa, x, vec, vecp, veca, o_w, o_b = _inputs(N, H, first)
    vo = torch.empty_like(veca)
    o, xo, vo = et_stack._oproj_epi(xa, o_w, o_b, x, vec, vecp, veca, vo)
    o_ref = torch.empty_like(o)
    kernels.gemm_group([(xa, o_w, True, o_b, o_ref, False)])
    x_ref, v_ref = et_stack._epilogue_fwd(x, vec, vecp, o_ref, veca)
    torch.cuda.synchronize()
    if H < 256:  # the same per-wave K slices and partial-sum order (the GEMM splits K = 256 16 ways)
        assert torch.equal(o, o_ref)
    assert _rel(o, o_ref) < 1e-6
    assert _rel(xo, x_ref) < 1e-6 and _rel(vo, v_ref) < 1e-6
    # and against a PyTorch restatement of the reference expressions
    ot = xa.double() @ o_w.double().t() + o_b.double()
    o1, o2, o3 = ot.split(H, dim=1)
    if first:
        xt, vt = x.double() + o3, veca.double()
    else:
        v1, v2, v3 = vecp.double().split(H, dim=2)
        xt = x.double() + (v1 * v2).sum(1) * o2 + o3
        vt = vec.double() + v3 * o1.unsqueeze(1) + veca.double()
    assert _rel(o, ot) < 1e-5 and _rel(xo, xt) < 1e-5 and _rel(vo, vt) < 1e-5


@pytest.mark.parametrize("N,H,with_vec", [(678, 128, True), (678, 128, False), (37, 64, True), (100, 256, True),
                                          (1, 128, True)])
def test_ln_mix_matches_layer_norm_and_linears(N, H, with_vec):
    from torchmdnet import et_stack
    g = torch.Generator().manual_seed(1)
    r = lambda *s: torch.randn(*s, generator=g).to(DEV)  # noqa: E731
    x = r(N, H) * 3 + 1.5  # an offset mean: the two-pass variance matters
    ln_w, ln_b = r(H), r(H)
    w, b = r(5 * H, H) / H ** 0.5, r(5 * H)
    vec = r(N, 3, H) if with_vec else None
    vec_w = r(3 * H, H) / H ** 0.5
    xn = torch.empty_like(x)
    qkv, vecp, xn, mean, rstd = et_stack._ln_mix(x, ln_w, ln_b, w, b, vec, vec_w, xn)
    torch.cuda.synchronize()
    xd = x.double()
    m = xd.mean(1, keepdim=True)
    var = ((xd - m) ** 2).mean(1, keepdim=True)
    rs = 1 / torch.sqrt(var + 1e-5)
    xn_ref = (xd - m) * rs * ln_w.double() + ln_b.double()
    assert _rel(mean, m) < 1e-6 and _rel(rstd, rs) < 1e-6
    assert _rel(xn, xn_ref) < 1e-6
    assert _rel(qkv, xn_ref @ w.double().t() + b.double()) < 1e-5
    # the stand-alone LayerNorm kernel gives the same xn / stats to fp32 reassociation
    _, _, xn0, mean0, rstd0 = et_stack._epi_ln(x, None, None, None, None, ln_w, ln_b)
    assert _rel(xn, xn0) < 1e-6 and _rel(mean, mean0) < 1e-6 and _rel(rstd, rstd0) < 1e-6
    if with_vec:
        vr = vec.double().reshape(3 * N, H) @ vec_w.double().t()
        assert _rel(vecp.reshape(3 * N, 3 * H), vr) < 1e-5
    else:
        assert vecp is None


@pytest.mark.parametrize("N,first,res", [(678, False, True), (678, True, True), (37, False, False), (1, False, True)])
def test_lnbwd_oproj_matches_two_launch_form(N, first, res):
    """tmdnet_et_lnbwd_oproj_f32 against tmdnet_ln_bwd_epilogue + the o_proj input-gradient GEMM."""
    from torchmdnet import et_stack, kernels
    H = 128
    g = torch.Generator().manual_seed(3)
    r = lambda *s: torch.randn(*s, generator=g).to(DEV)  # noqa: E731
    g_xn, x, ln_w = r(N, H), r(N, H) * 2 + 0.7, r(H)
    g_res = r(N, H) if res else None
    g_vec = r(N, 3, H)
    vecp = None if first else r(N, 3, 3 * H)
    o = r(N, 3 * H)
    o_w = r(3 * H, H) / H ** 0.5
    xd = x.double()
    mean = xd.mean(1, keepdim=True)
    rstd = 1 / torch.sqrt(((xd - mean) ** 2).mean(1, keepdim=True) + 1e-5)
    mean, rstd = mean.float(), rstd.float()
    gvp1, go1 = torch.full((N, 3, 3 * H), 7.0, device=DEV), torch.empty((N, 3 * H), device=DEV)
    gx1, gxa1 = et_stack._ln_bwd_oproj(g_xn, x, mean, rstd, ln_w, g_res, g_vec, vecp, o, o_w, gvp1, go1)
    gvp0, go0 = torch.full((N, 3, 3 * H), 7.0, device=DEV), torch.empty((N, 3 * H), device=DEV)
    gx0 = et_stack._ln_bwd_epi(g_xn, x, mean, rstd, ln_w, g_res, g_vec, vecp, o, gvp0, go0)
    gxa0 = torch.empty((N, H), device=DEV)
    kernels.gemm_group([(go0, o_w, False, None, gxa0, False)])
    torch.cuda.synchronize()
    assert _rel(gx1, gx0) < 1e-5 and _rel(go1, go0) < 1e-5 and _rel(gxa1, gxa0) < 1e-5
    if not first:
        assert _rel(gvp1, gvp0) < 1e-5
    # fp64 restatement of the LayerNorm backward (torch.native_layer_norm_backward's formula)
    xh = (xd - mean.double()) * rstd.double()
    gh = g_xn.double() * ln_w.double()
    gx_ref = rstd.double() * (gh - gh.mean(1, keepdim=True) - xh * (gh * xh).mean(1, keepdim=True))
    if res:
        gx_ref = gx_ref + g_res.double()
    assert _rel(gx1, gx_ref) < 1e-5


def _c2_model():
    from torchmdnet.models.model import create_model
    args = yaml_args("equivariant-transformer", embedding_dimension=128, num_layers=8, num_rbf=64, num_heads=8,
                     derivative=True)
    torch.manual_seed(0)
    return create_model(args), args


def test_c2_model_node_fused_vs_three_launch_and_oracle(monkeypatch):
    """Energies / forces of the C2 workload with the node-fused forward against the three-launch form and
    the fp64 oracle (north_star: energies and forces 1e-4 relative), and the fused launches really ran."""
    from oracle import model_oracle as O
    from torchmdnet import et_stack
    calls = []
    orig = et_stack._ln_mix
    monkeypatch.setattr(et_stack, "_ln_mix", lambda *a, **k: (calls.append(1), orig(*a, **k))[1])
    m, args = _c2_model()
    z, pos, batch = O.qm9_like(32)
    y_ref, f_ref = O.energy_forces(m.state_dict(), dict(args), z, pos, batch)
    m = m.to(DEV)
    monkeypatch.setattr(et_stack, "NODE_FUSE", True)
    y, f = m(z.to(DEV), pos.float().to(DEV), batch.to(DEV))
    assert len(calls) == 8
    monkeypatch.setattr(et_stack, "NODE_FUSE", False)
    y0, f0 = m(z.to(DEV), pos.float().to(DEV), batch.to(DEV))
    assert len(calls) == 8
    assert _rel(y.detach(), y0.detach()) < 1e-5 and _rel(f.detach(), f0.detach()) < 1e-4
    assert _rel(y.detach().cpu(), y_ref.detach()) < 1e-4 and _rel(f.detach().cpu(), f_ref) < 1e-4


def test_c2_force_loss_gradients_node_fused_vs_three_launch(monkeypatch):
    """The training step's force-matching parameter gradients (second order through the saved forward
    activations the fused kernels produce: xn, mean / rstd, o, x, vec) with the fusion on and off."""
    from oracle import model_oracle as O
    from torchmdnet import et_stack
    m, _ = _c2_model()
    m = m.to(DEV)
    z, pos, batch = O.qm9_like(8)
    z, pos, batch = z.to(DEV), pos.float().to(DEV), batch.to(DEV)

    def grads(on):
        monkeypatch.setattr(et_stack, "NODE_FUSE", on)
        m.zero_grad(set_to_none=True)
        y, f = m(z, pos, batch)
        (y.pow(2).sum() + f.pow(2).sum()).backward()
        return {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}

    a, b = grads(True), grads(False)
    assert a.keys() == b.keys()
    for n in a:
        assert _rel(a[n], b[n]) < 5e-5, n


def test_c2_graph_replay_node_fused(monkeypatch):
    """The bench's execution form: a captured HIP graph of the node-fused evaluation replays to the eager
    result."""
    from oracle import model_oracle as O
    from torchmdnet import et_stack
    from torchmdnet.graphs import GraphedEnergyForces
    monkeypatch.setattr(et_stack, "NODE_FUSE", True)
    m, _ = _c2_model()
    m = m.to(DEV)
    z, pos, batch = O.qm9_like(32)
    z, pos, batch = z.to(DEV), pos.float().to(DEV), batch.to(DEV)
    y0, f0 = m(z, pos, batch)
    gm = GraphedEnergyForces(m, z, pos, batch)
    y1, f1 = gm(pos)
    torch.cuda.synchronize()
    assert _rel(y1, y0.detach()) < 1e-5 and _rel(f1, f0.detach()) < 1e-5
    gm.release()
