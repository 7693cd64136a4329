"""Reference edge cases on the GPU path (ports of the reference's own tests + reference-run fixtures).

* lower cutoff: tests/test_model_utils.py:9-60 (pair counts around cutoff_lower / cutoff_upper)
  through OptimizedDistance, and a whole ET model with cutoff_lower = 2 A against the fixture
  tests/golden/et_tiny_cl2_f64.npz produced by the reference (shifted CosineCutoff,
  models/utils.py:362-390; neighbour lower bound);
* the isolated-atom force loss: tests/test_model_utils.py:87-104 (no NaN in d(sum F)/d(embedding)
  when one atom has no neighbour: the head's zero-norm guard, utils.py:500-512);
* the Atomref prior of ET-QM9.yaml (priors/atomref.py:8-42) with non-zero per-element values
  against tests/golden/et_tiny_atomref_f64.npz (outputs and force-loss double backward).
"""
import numpy as np
import pytest
import torch

from conftest import golden, state_dict_from, yaml_args

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _lib_loaded():
    from torchmdnet import _native
    _native.load()
    assert "libtmdnet_hip.so" in open("/proc/self/maps").read()


@pytest.mark.parametrize("cutoff_lower", [0, 2])
@pytest.mark.parametrize("cutoff_upper", [5, 10])
@pytest.mark.parametrize("return_vecs", [False, True])
@pytest.mark.parametrize("loop", [False, True])
def test_distance_calculation(cutoff_lower, cutoff_upper, return_vecs, loop):
    from torchmdnet.models.utils import OptimizedDistance
    _lib_loaded()
    dist = OptimizedDistance(cutoff_lower, cutoff_upper, max_num_pairs=-100, return_vecs=return_vecs, loop=loop)
    batch = torch.tensor([0, 0], device=DEV)
    loop_extra = len(batch) if loop else 0
    # two atoms, distance between lower and upper cutoff
    pos = torch.tensor([[0, 0, 0], [(cutoff_lower + cutoff_upper) / 2, 0, 0]], dtype=torch.float, device=DEV)
    edge_index, edge_weight, edge_vec = dist(pos, batch)
    assert edge_index.size(1) == 2 + loop_extra
    if return_vecs:
        assert edge_vec is not None
    # two atoms closer than the lower cutoff
    if cutoff_lower > 0:
        pos = torch.tensor([[0, 0, 0], [cutoff_lower / 2, 0, 0]], dtype=torch.float, device=DEV)
        edge_index, _, _ = dist(pos, batch)
        assert edge_index.size(1) == loop_extra
    # two atoms beyond the upper cutoff
    pos = torch.tensor([[0, 0, 0], [cutoff_upper + 1, 0, 0]], dtype=torch.float, device=DEV)
    edge_index, _, _ = dist(pos, batch)
    assert edge_index.size(1) == loop_extra
    # many atoms in a unit cube: all pairs (cl = 0) or only self loops (cl = 2)
    batch = torch.zeros(100, dtype=torch.long, device=DEV)
    pos = torch.rand(100, 3, device=DEV)
    edge_index, _, _ = dist(pos, batch)
    loop_extra = len(batch) if loop else 0
    if cutoff_lower > 0:
        assert edge_index.size(1) == loop_extra
    else:
        assert edge_index.size(1) == len(batch) * (len(batch) - 1) + loop_extra


@pytest.mark.parametrize("cl", [0.0, 2.0])
def test_edge_geometry_lower_cutoff_matches_formula(cl):
    """The fused edge-geometry kernel's CosineCutoff(cl, cu) and expnorm RBF (reference
    models/utils.py:322-344, 362-390) against the formulas in fp64, r sweeping both cutoffs."""
    from torchmdnet import kernels
    from oracle import model_oracle as O
    cu, R = 5.0, 16
    r = torch.linspace(0.05, 6.0, 997, dtype=torch.float64)
    n = r.numel()
    pos = torch.zeros(2 * n, 3, dtype=torch.float64)
    pos[1::2, 0] = r  # pairs (2i, 2i+1), one molecule each
    batch = torch.arange(n).repeat_interleave(2)
    g = kernels.build_graph(pos.to(DEV), batch.to(DEV), cl, cu, 4 * n, loop=True)
    start = np.exp(-cu + cl)
    means = torch.linspace(start, 1.0, R, dtype=torch.float64)
    betas = torch.full((R,), (2.0 / R * (1 - start)) ** -2, dtype=torch.float64)
    f, C, _ = kernels._EdgeGeom.apply(g.deltas, g.distances, g, means.to(DEV), betas.to(DEV), cl, cu,
                                      kernels.nat.RBF_EXPNORM, (True, True, True))
    d = g.distances.detach().cpu()
    assert torch.allclose(C.cpu(), O.cosine_cutoff(d, cl, cu), rtol=1e-12, atol=1e-14)
    assert torch.allclose(f.cpu(), O.expnorm(d, means, betas, cl, cu), rtol=1e-12, atol=1e-14)
    nonself = (g.src != g.dst).cpu()
    inside = (r >= cl) & (r < cu)
    assert int(nonself.sum()) == 2 * int(inside.sum())  # the neighbour list's [cl, cu) window


def _model_from_fixture(d, **kw):
    from torchmdnet.models.model import create_model
    args = yaml_args("equivariant-transformer", embedding_dimension=32, num_layers=2, num_rbf=16, num_heads=4,
                     max_num_neighbors=32, derivative=True, output_model="Scalar", precision=64, **kw)
    m = create_model(args)
    m.load_state_dict({k: torch.tensor(v) for k, v in state_dict_from(d).items()})
    return m.to(DEV)


@pytest.mark.parametrize("name,kw", [("et_tiny_cl2_f64", dict(cutoff_lower=2.0, cutoff_upper=5.0)),
                                     ("et_tiny_atomref_f64", dict(prior_model="Atomref",
                                                                  prior_args={"max_z": 100})),
                                     # non-SiLU activations: the kernels' TMDNET_ET_ACT codes, first and
                                     # second order (the hand-written force-loss backward included)
                                     ("et_tiny_act_tanh_ssp_f64", dict(activation="tanh", attn_activation="ssp")),
                                     ("et_tiny_act_sigmoid_tanh_f64",
                                      dict(activation="sigmoid", attn_activation="tanh"))])
def test_et_edge_case_fixture(name, kw):
    _lib_loaded()
    d = golden(name + ".npz")
    m = _model_from_fixture(d, **kw)
    pos = torch.tensor(d["pos"], device=DEV)
    y, neg_dy = m(torch.tensor(d["z"], device=DEV), pos, torch.tensor(d["batch"], device=DEV))
    assert np.allclose(y.detach().cpu().numpy(), d["y"], rtol=1e-9, atol=1e-10)
    assert np.allclose(neg_dy.detach().cpu().numpy(), d["neg_dy"], rtol=1e-9, atol=1e-9)
    loss = (y ** 2).sum() + (neg_dy ** 2).sum()
    named = [(n, p) for n, p in m.named_parameters() if p.requires_grad]
    grads = torch.autograd.grad(loss, [p for _, p in named], allow_unused=True)
    for (n, _), g in zip(named, grads):
        ref = d["g2/" + n]
        got = np.zeros_like(ref) if g is None else g.detach().cpu().numpy()
        assert np.allclose(got, ref, rtol=1e-7, atol=1e-9), n


def test_gated_eq_gradients_isolated_atom():
    """Reference tests/test_model_utils.py:87-104: one atom outside every other atom's cutoff; the
    gradient of the forces w.r.t. the embedding has no NaN."""
    from torchmdnet.models.model import create_model
    _lib_loaded()
    torch.manual_seed(0)
    model = create_model(yaml_args("equivariant-transformer", cutoff_upper=5, derivative=True)).to(DEV)
    z = torch.tensor([1, 1, 8], device=DEV)
    pos = torch.tensor([[0, 0, 0], [0, 1, 0], [10, 0, 0]], dtype=torch.float, device=DEV)
    _, forces = model(z, pos)
    emb = model.representation_model.embedding.weight
    (deriv,) = torch.autograd.grad(forces.sum(), emb, retain_graph=True)
    assert not deriv.isnan().any()  # (sum F = 0 by translation invariance: this gradient is 0)
    (deriv2,) = torch.autograd.grad(forces.pow(2).sum(), emb)  # a force loss that does depend on it
    assert torch.isfinite(deriv2).all() and deriv2.abs().sum() > 0


@pytest.mark.parametrize("R", [16, 32, 50, 64])
@pytest.mark.parametrize("rbf", ["expnorm", "gauss"])
@pytest.mark.parametrize("dtype,tol", [(torch.float64, 1e-11), (torch.float32, 2e-5)])
@pytest.mark.parametrize("slots", [1, 3])
def test_edge_geometry_backward_matches_autograd(R, rbf, dtype, tol, slots):
    """tmdnet_edge_geom_bwd_multi (the lane-parallel k_bwd_v: R = 16 / 32 / 64; R = 50 takes the
    wave-per-edge form) against autograd of the formulas (reference models/utils.py:272-390, the unit
    vectors torchmd_et.py:173-174): g_r and g_deltas for 1 or 3 gradient slots of rbf and cutoff, with
    self loops and a lower cutoff."""
    from torchmdnet import kernels
    from oracle import model_oracle as O
    cl, cu = 0.5, 5.0
    g = torch.Generator().manual_seed(R + slots)
    pos = torch.randn(300, 3, generator=g, dtype=torch.float64) * 2.0
    batch = torch.arange(6).repeat_interleave(50)
    gr = kernels.build_graph(pos.to(dtype).to(DEV), batch.to(DEV), cl, cu, 300 * 300, loop=True)
    E = gr.num_pairs
    if rbf == "expnorm":
        start = np.exp(-cu + cl)
        mu = torch.linspace(start, 1.0, R, dtype=torch.float64)
        beta = torch.full((R,), (2.0 / R * (1 - start)) ** -2, dtype=torch.float64)
        code = kernels.nat.RBF_EXPNORM
    else:
        mu = torch.linspace(cl, cu, R, dtype=torch.float64)
        beta = torch.full((1,), -0.5 / float(mu[1] - mu[0]) ** 2, dtype=torch.float64)
        code = kernels.nat.RBF_GAUSS
    dl = gr.deltas.detach().clone().requires_grad_(True)
    r = gr.distances.detach().clone().requires_grad_(True)
    outs = kernels._EdgeGeom.apply(dl, r, gr, mu.to(dtype).to(DEV), beta.to(dtype).to(DEV), cl, cu, code,
                                   (True, True, True), None, (slots, slots))
    f, C, u = outs[:3]
    gens = [torch.randn(t.shape, generator=g, dtype=torch.float64) for t in outs]
    loss = sum((t * w.to(dtype).to(DEV)).sum() for t, w in zip(outs, gens))
    g_dl, g_r = torch.autograd.grad(loss, [dl, r])
    # composite in fp64 on the CPU
    dl64 = gr.deltas.detach().double().cpu().requires_grad_(True)
    r64 = gr.distances.detach().double().cpu().requires_grad_(True)
    f64 = O.expnorm(r64, mu, beta, cl, cu) if rbf == "expnorm" else O.gauss(r64, mu, beta[0])
    C64 = O.cosine_cutoff(r64, cl, cu)
    self_e = (gr.src == gr.dst).cpu().unsqueeze(1)
    nrm = torch.where(self_e, torch.ones_like(r64).unsqueeze(1), dl64.norm(dim=1, keepdim=True))
    u64 = torch.where(self_e, dl64, dl64 / nrm)
    outs64 = [f64, C64, u64] + [f64] * (slots - 1) + [C64] * (slots - 1)
    loss64 = sum((t * w).sum() for t, w in zip(outs64, gens))
    e_dl, e_r = torch.autograd.grad(loss64, [dl64, r64])
    assert E > 1000
    rel = lambda a, b: float((a.double().cpu() - b).abs().max() / b.abs().max().clamp_min(1e-30))  # noqa: E731
    assert rel(g_r, e_r) < tol, rel(g_r, e_r)
    assert rel(g_dl, e_dl) < tol, rel(g_dl, e_dl)


@pytest.mark.parametrize("dtype,tol", [(torch.float64, 1e-11), (torch.float32, 2e-5)])
@pytest.mark.parametrize("slots", [1, 2])
def test_edge_geometry_backward_without_rbf_gradient(dtype, tol, slots):
    """No consumer sends an rbf-row gradient (the fused C5 stack and neighbour embedding return g_r
    themselves): the thread-per-edge k_bwd_e form -- cutoff and unit-vector terms only -- against autograd of
    the formulas, with self loops and a lower cutoff."""
    from torchmdnet import kernels
    cl, cu, R = 0.5, 5.0, 64
    g = torch.Generator().manual_seed(11 + slots)
    pos = torch.randn(300, 3, generator=g, dtype=torch.float64) * 2.0
    batch = torch.arange(6).repeat_interleave(50)
    gr = kernels.build_graph(pos.to(dtype).to(DEV), batch.to(DEV), cl, cu, 300 * 300, loop=True)
    start = np.exp(-cu + cl)
    mu = torch.linspace(start, 1.0, R, dtype=torch.float64)
    beta = torch.full((R,), (2.0 / R * (1 - start)) ** -2, dtype=torch.float64)
    dl = gr.deltas.detach().clone().requires_grad_(True)
    r = gr.distances.detach().clone().requires_grad_(True)
    outs = kernels._EdgeGeom.apply(dl, r, gr, mu.to(dtype).to(DEV), beta.to(dtype).to(DEV), cl, cu,
                                   kernels.nat.RBF_EXPNORM, (True, True, True), None, (1, slots))
    C_all = [outs[1]] + list(outs[3:])
    u = outs[2]
    gens = [torch.randn(t.shape, generator=g, dtype=torch.float64) for t in C_all + [u]]
    loss = sum((t * w.to(dtype).to(DEV)).sum() for t, w in zip(C_all + [u], gens))  # f unused: no gradient
    g_dl, g_r = torch.autograd.grad(loss, [dl, r])
    from oracle import model_oracle as O
    dl64 = gr.deltas.detach().double().cpu().requires_grad_(True)
    r64 = gr.distances.detach().double().cpu().requires_grad_(True)
    C64 = O.cosine_cutoff(r64, cl, cu)
    self_e = (gr.src == gr.dst).cpu().unsqueeze(1)
    nrm = torch.where(self_e, torch.ones_like(r64).unsqueeze(1), dl64.norm(dim=1, keepdim=True))
    u64 = torch.where(self_e, dl64, dl64 / nrm)
    loss64 = sum((t * w).sum() for t, w in zip([C64] * slots + [u64], gens))
    e_dl, e_r = torch.autograd.grad(loss64, [dl64, r64])
    rel = lambda a, b: float((a.double().cpu() - b).abs().max() / b.abs().max().clamp_min(1e-30))  # noqa: E731
    assert rel(g_r, e_r) < tol, rel(g_r, e_r)
    assert rel(g_dl, e_dl) < tol, rel(g_dl, e_dl)
