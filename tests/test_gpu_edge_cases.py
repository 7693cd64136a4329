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
