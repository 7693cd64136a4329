"""GPU checks of the fused dk/dv projection edge kernels (csrc/et_fused.hip, "FEP"): the ET message with
the projection (reference torchmd_et.py:282-291) evaluated on the fp16 MFMA inside the edge kernel from
the distances (the RBF of models/utils.py:272-344 formed in registers), on planar-layout graphs -- the
forward and the force pass's backward (d pre / d r = W f'(r) on the MFMA, contracted in-kernel).

Bars: the fused fp32 model against the SAME weights in fp64 (no fusion at fp64): energies 1e-5, forces
1e-4 relative (max-abs error over max |value|: the north_star bar; the unfused fp32 path sits at
~7e-5 on this box), and the same against the unfused fp32 path."""
import pytest
import torch

from conftest import yaml_args

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return float((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30))


def _water_box(n, seed=7):
    g = torch.Generator().manual_seed(seed)
    L = (n / 0.1003) ** (1.0 / 3.0)
    pos = torch.rand(n, 3, generator=g, dtype=torch.float64) * L
    z = torch.tensor([8, 1, 1], dtype=torch.long).repeat(n // 3 + 1)[:n]
    return z, pos, L


def _model(R, rbf_type, cl=0.0, precision=32):
    from torchmdnet.models.model import create_model
    torch.manual_seed(0)
    m = create_model(yaml_args("equivariant-transformer", embedding_dimension=128, num_layers=3, num_rbf=R,
                               num_heads=8, max_num_neighbors=128, derivative=True, output_model="Scalar",
                               rbf_type=rbf_type, cutoff_lower=cl, precision=precision))
    return m


def _run(m, z, pos, L, dtype):
    m = m.to(DEV)
    d = m.representation_model.distance
    d.box = torch.eye(3, dtype=dtype) * L
    d.use_periodic = True
    d.strategy = "cell"
    y, f = m(z.to(DEV), pos.to(dtype).to(DEV), torch.zeros_like(z).to(DEV))
    return y.detach(), None if f is None else f.detach()


@pytest.mark.parametrize("R,rbf_type,cl", [(64, "expnorm", 0.0), (32, "expnorm", 0.0), (64, "gauss", 0.0),
                                           (64, "expnorm", 0.5)])
def test_fused_forward_matches_fp64_and_unfused(R, rbf_type, cl, monkeypatch):
    from torchmdnet import et_stack, kernels
    calls, bcalls = [], []
    orig, origb = kernels.et_fused_fwd_launch, kernels.et_fused_bwd_launch

    def counting(*a, **k):
        calls.append(1)
        return orig(*a, **k)

    def counting_b(*a, **k):
        bcalls.append(1)
        return origb(*a, **k)

    monkeypatch.setattr(kernels, "et_fused_fwd_launch", counting)
    monkeypatch.setattr(kernels, "et_fused_bwd_launch", counting_b)
    monkeypatch.setattr(et_stack, "FEP_BWD", "fused")
    monkeypatch.setattr(et_stack, "FUSED_BWD", True)
    z, pos, L = _water_box(3000)
    m = _model(R, rbf_type, cl)
    sd = m.state_dict()
    y, f = _run(m, z, pos, L, torch.float32)
    assert len(calls) == 3 and len(bcalls) == 3, "the fused kernels did not run"  # one per layer each
    m64 = _model(R, rbf_type, cl, precision=64)
    m64.load_state_dict({k: v.double() if v.is_floating_point() else v for k, v in sd.items()})
    y64, f64 = _run(m64, z, pos, L, torch.float64)
    assert _rel(y, y64) < 1e-5
    assert _rel(f, f64) < 1e-4
    # the fused forward with the unfused force-pass backward over rows formed by the GEMM ("lazy")
    monkeypatch.setattr(et_stack, "FUSED_BWD", False)
    monkeypatch.setattr(et_stack, "FEP_BWD", "lazy")
    y1, f1 = _run(m, z, pos, L, torch.float32)
    assert len(bcalls) == 3 and len(calls) == 6
    assert _rel(y, y1) < 1e-5
    assert _rel(f, f1) < 1e-4
    # "off": with a backward to follow the forward is the unfused one; energy only -> fused
    monkeypatch.setattr(et_stack, "FEP_BWD", "off")
    n0 = len(calls)
    y2, f2 = _run(m, z, pos, L, torch.float32)
    assert len(calls) == n0
    assert _rel(y, y2) < 1e-5 and _rel(f, f2) < 1e-4
    m.derivative = False
    with torch.no_grad():
        y3, _ = _run(m, z, pos, L, torch.float32)
    m.derivative = True
    assert len(calls) == n0 + 3
    assert _rel(y, y3) < 1e-5
    monkeypatch.setattr(et_stack, "FEP", "0")
    n0 = len(calls)
    y0, f0 = _run(m, z, pos, L, torch.float32)
    assert len(calls) == n0
    assert _rel(y, y0) < 1e-5
    assert _rel(f, f0) < 1e-4


@pytest.mark.parametrize("planar", [False, True])
def test_fused_c2_molecules_vs_oracle_and_unfused(planar, monkeypatch):
    """The fused kernels on the C2 workload (32 QM9-like molecules, 128 ch, 8 layers, 64 RBF): the
    reference per-head [x|v1|v2] v layout (default below the planar threshold) and the planar one,
    against the fp64 oracle and the unfused path (TMDNET_FEP=0), energies and forces."""
    from oracle import model_oracle as O
    from torchmdnet import et_stack, kernels
    from torchmdnet.models.model import create_model
    calls = []
    orig, origb = kernels.et_fused_fwd_launch, kernels.et_fused_bwd_launch
    monkeypatch.setattr(kernels, "et_fused_fwd_launch", lambda *a, **k: (calls.append("f"), orig(*a, **k))[1])
    monkeypatch.setattr(kernels, "et_fused_bwd_launch", lambda *a, **k: (calls.append("b"), origb(*a, **k))[1])
    monkeypatch.setattr(et_stack, "FEP_MIN_EDGES", 0)
    if planar:
        monkeypatch.setattr(et_stack, "PLANAR_MIN_EDGES", 0)
    args = yaml_args("equivariant-transformer", embedding_dimension=128, num_layers=8, num_rbf=64, num_heads=8,
                     derivative=True)
    torch.manual_seed(0)
    m = create_model(args)
    z, pos, batch = O.qm9_like(32)
    y_ref, f_ref = O.energy_forces(m.state_dict(), dict(args), z, pos, batch)
    m = m.to(DEV)
    y, f = m(z.to(DEV), pos.float().to(DEV), batch.to(DEV))
    assert calls.count("f") == 8 and calls.count("b") == 8, calls
    assert _rel(y.detach().cpu(), y_ref.detach()) < 1e-4
    assert _rel(f.detach().cpu(), f_ref) < 1e-4
    monkeypatch.setattr(et_stack, "FEP", "0")
    y0, f0 = m(z.to(DEV), pos.float().to(DEV), batch.to(DEV))
    assert calls.count("f") == 8
    assert _rel(y.detach(), y0.detach()) < 1e-5
    assert _rel(f.detach(), f0.detach()) < 1e-4


def test_fused_neighbor_embedding_force_pass_and_parameter_gradients(monkeypatch):
    """The neighbour embedding with distance_proj fused into its aggregation kernel
    (kernels.nbr_embed_fused: tmdnet_nbr_fused_fwd_f32, dr-mode tmdnet_nbr_fused_bwd_f32; reference
    utils.py:90-108) on a 3000-atom periodic water box: energy and forces against the row path
    (TMDNET_NE_FUSED=0: W = distance_proj(rbf) rows, the unfused kernels) and against fp64; then the
    composite backward (parameter gradients of an energy loss, distance_proj / embedding / combine)
    against the row path's."""
    from torchmdnet import kernels
    from torchmdnet.models import torchmd_et
    calls = []
    orig = kernels.nbr_embed_fused
    monkeypatch.setattr(kernels, "nbr_embed_fused", lambda *a, **k: (calls.append(1), orig(*a, **k))[1])
    z, pos, L = _water_box(3000)
    m = _model(64, "expnorm")
    sd = m.state_dict()
    y, f = _run(m, z, pos, L, torch.float32)
    assert len(calls) == 1, "the fused neighbour embedding did not run"
    monkeypatch.setattr(torchmd_et, "NE_FUSED", False)
    y0, f0 = _run(m, z, pos, L, torch.float32)
    assert len(calls) == 1
    assert _rel(y, y0) < 1e-5 and _rel(f, f0) < 1e-4
    m64 = _model(64, "expnorm", precision=64)
    m64.load_state_dict({k: v.double() if v.is_floating_point() else v for k, v in sd.items()})
    y64, f64 = _run(m64, z, pos, L, torch.float64)
    assert _rel(y, y64) < 1e-5 and _rel(f, f64) < 1e-4

    monkeypatch.setattr(torchmd_et, "NE_FUSED", True)
    m.derivative = False
    m.zero_grad(set_to_none=True)
    m = m.to(DEV)
    dd = m.representation_model.distance
    dd.box = torch.eye(3) * L
    dd.use_periodic = True
    dd.strategy = "cell"
    n0 = len(calls)
    m(z.to(DEV), pos.float().to(DEV), torch.zeros_like(z).to(DEV))[0].sum().backward()
    assert len(calls) == n0 + 1
    ne = m.representation_model.neighbor_embedding
    g1 = [p.grad.detach().clone() for p in (ne.distance_proj.weight, ne.distance_proj.bias, ne.embedding.weight,
                                             ne.combine.weight)]
    monkeypatch.setattr(torchmd_et, "NE_FUSED", False)
    m.zero_grad(set_to_none=True)
    m(z.to(DEV), pos.float().to(DEV), torch.zeros_like(z).to(DEV))[0].sum().backward()
    g0 = [p.grad for p in (ne.distance_proj.weight, ne.distance_proj.bias, ne.embedding.weight, ne.combine.weight)]
    m.derivative = True
    for a, b in zip(g1, g0):
        assert _rel(a, b) < 1e-4


def test_fused_neighbor_embedding_force_loss_second_order(monkeypatch):
    """Force-matching training through the fused neighbour embedding: the dr-mode backward
    (_NbrEmbedFusedBwd) differentiated again (its composite second order) gives the same parameter
    gradients of a force loss as the row path (TMDNET_NE_FUSED=0)."""
    from torchmdnet.models import torchmd_et
    z, pos, L = _water_box(3000)
    m = _model(64, "expnorm").to(DEV)
    d = m.representation_model.distance
    d.box = torch.eye(3) * L
    d.use_periodic = True
    d.strategy = "cell"
    ne = m.representation_model.neighbor_embedding
    ps = [ne.distance_proj.weight, ne.distance_proj.bias, ne.embedding.weight, ne.combine.weight]

    def grads(fused):
        monkeypatch.setattr(torchmd_et, "NE_FUSED", fused)
        m.zero_grad(set_to_none=True)
        y, f = m(z.to(DEV), pos.float().to(DEV), torch.zeros_like(z).to(DEV))
        (f.pow(2).sum() + y.sum()).backward()
        return [p.grad.detach().clone() for p in ps]

    g1, g0 = grads(True), grads(False)
    for a, b in zip(g1, g0):
        assert _rel(a, b) < 1e-4
