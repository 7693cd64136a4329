"""The large-system periodic model path against the fp64 oracle (VERDICT r3 "next" #1).

C5 (the 50k-atom water box) is too large for any CPU oracle, so the switches that only large systems
turn on are FORCED here on a 1000-2000-atom periodic water box that the oracle (oracle/model_oracle.py,
pinned to the reference by tests/golden) finishes in seconds:

* ``strategy="cell"`` with a rectangular box (reference neighbors_cuda_cell.cuh; minimum image
  neighbors_cpu.cpp:63-70 on the oracle side);
* Morton renumbering of the atoms (``kernels.REORDER_MIN_ATOMS`` -> 0; torchmd_et.py forward);
* planar v / dv rows (``et_stack.PLANAR_MIN_EDGES`` -> 0), which also enables the fused-projection
  forward (et_fused.hip) for energy-only calls;
* pair-shared projection rows (always on for symmetric lists);
* the merged dr-mode force backward ``k_bwd_merged`` (``TUNE_ET_MERGED_MIN_NODES`` -> 0), with the
  pair-symmetry precondition of its source role checked on the device before every launch
  (``kernels.CHECK_SYMMETRY``).

Compared: fp32 energies and forces against ``O.energy_forces(..., box=L*I)`` in fp64 (bar 1e-4,
max-abs error over max |value|: the north_star bar), the energy-only fused forward, force-loss
parameter gradients (the reference LNNP.step objective, double backward), and TensorNet on a periodic
box (static_shapes off -- Morton renumbering -- and on -- the CUDA padding semantics)."""
import numpy as np
import pytest
import torch

from conftest import yaml_args
from oracle import model_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 1e-4


def _rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _water_box(n, seed=11):
    g = torch.Generator().manual_seed(seed)
    L = (n / 0.1003) ** (1.0 / 3.0)
    pos = torch.rand(n, 3, generator=g, dtype=torch.float64) * L
    z = torch.tensor([8, 1, 1], dtype=torch.long).repeat(n // 3 + 1)[:n]
    return z, pos, torch.zeros(n, dtype=torch.long), L


@pytest.fixture
def large_switches(monkeypatch):
    """Every large-system launch form on, whatever the size."""
    from torchmdnet import et_stack, kernels
    monkeypatch.setattr(kernels, "REORDER_MIN_ATOMS", 0)
    monkeypatch.setattr(et_stack, "PLANAR_MIN_EDGES", 0)
    monkeypatch.setattr(kernels, "CHECK_SYMMETRY", True)
    prev = kernels.set_tuning(kernels.TUNE_ET_MERGED_MIN_NODES, 0)
    merged = []
    orig = kernels.et_message_bwd_launch

    def spy(*a, **k):
        if k.get("g_r") is not None:
            merged.append(1)
        return orig(*a, **k)

    monkeypatch.setattr(kernels, "et_message_bwd_launch", spy)
    yield merged
    kernels.set_tuning(kernels.TUNE_ET_MERGED_MIN_NODES, prev)


def _et(layers=8, precision=32):
    from torchmdnet.models.model import create_model
    torch.manual_seed(0)
    return create_model(yaml_args("equivariant-transformer", embedding_dimension=128, num_layers=layers,
                                  num_rbf=64, num_heads=8, cutoff_upper=5.0, max_num_neighbors=128,
                                  derivative=True, precision=precision))


def _periodic(m, L, dtype=torch.float32):
    d = m.representation_model.distance
    d.box = torch.eye(3, dtype=dtype) * L
    d.use_periodic = True
    d.strategy = "cell"
    return m


def _cfg(args, L):
    cfg = dict(args)
    cfg["box"] = np.eye(3) * L
    return cfg


@pytest.mark.parametrize("path", ["rows", "fused"])
def test_et_periodic_box_vs_oracle(path, large_switches, monkeypatch):
    """ET (128 ch, 8 layers, 64 RBF, 8 heads, cutoff 5) on a 2000-atom periodic water box with every
    large-system switch forced: energy and forces vs the fp64 oracle, through the pair-row path (merged
    dr-mode backward ``k_bwd_merged``) and through the fused-projection kernels (et_fused.hip, the C5
    default); the energy-only call runs the fused forward and matches too."""
    from torchmdnet import et_stack, kernels
    fused_b = []
    if path == "fused":
        monkeypatch.setattr(et_stack, "FEP_MIN_EDGES", 0)
        orig_b = kernels.et_fused_bwd_launch
        monkeypatch.setattr(kernels, "et_fused_bwd_launch", lambda *a, **k: (fused_b.append(1), orig_b(*a, **k))[1])
    else:
        monkeypatch.setattr(et_stack, "FEP", "0")
    z, pos, batch, L = _water_box(2000)
    m = _et()
    y_ref, f_ref = O.energy_forces(m.state_dict(), _cfg(_args(), L), z, pos, batch)
    m = _periodic(m.to(DEV), L)
    y, f = m(z.to(DEV), pos.float().to(DEV), batch.to(DEV))
    if path == "rows":
        assert len(large_switches) == 8, "the dr-mode force backward did not run per layer"
    else:
        assert len(fused_b) == 8, "the fused force backward did not run per layer"
    assert _rel(y, y_ref) < TOL, _rel(y, y_ref)
    assert _rel(f, f_ref) < TOL, _rel(f, f_ref)
    # energy only (no backward follows): the fused dk/dv projection forward
    calls = []
    orig = kernels.et_fused_fwd_launch

    def counting(*a, **k):
        calls.append(1)
        return orig(*a, **k)

    monkeypatch.setattr(kernels, "et_fused_fwd_launch", counting)
    monkeypatch.setattr(et_stack, "FEP", "auto")
    monkeypatch.setattr(et_stack, "FEP_MIN_EDGES", 0)
    m.derivative = False
    with torch.no_grad():
        y0, _ = m(z.to(DEV), pos.float().to(DEV), batch.to(DEV))
    m.derivative = True
    assert len(calls) == 8, "the fused forward did not run"
    assert _rel(y0, y_ref) < TOL, _rel(y0, y_ref)


def _args():
    return yaml_args("equivariant-transformer", embedding_dimension=128, num_layers=8, num_rbf=64, num_heads=8,
                     cutoff_upper=5.0, max_num_neighbors=128, derivative=True)


def test_et_periodic_box_force_loss_gradients(large_switches):
    """Force-loss parameter gradients (reference LNNP.step: MSE(y) + MSE(neg_dy), double backward) of
    the periodic large-system path on a 1000-atom water box vs the fp64 oracle."""
    from test_gpu_train_parity import _compare, _oracle_grads
    from torchmdnet.training import LNNPStep
    z, pos, batch, L = _water_box(1000, seed=5)
    args = _args()
    m = _et()
    g = torch.Generator().manual_seed(9)
    y_t = torch.randn(1, 1, generator=g, dtype=torch.float64) * 10
    f_t = torch.randn(z.shape[0], 3, generator=g, dtype=torch.float64)
    loss_ref, ref = _oracle_grads(m, _cfg(args, L), z, pos, batch, y_t, f_t, 0.05, 0.95)
    m = _periodic(m.to(DEV), L)
    tr = LNNPStep(m, lr=0.0, y_weight=0.05, neg_dy_weight=0.95)
    tr.opt.zero_grad(set_to_none=False)
    lt = tr.loss(z.to(DEV), pos.float().to(DEV), batch.to(DEV), y_t.float().to(DEV), f_t.float().to(DEV))
    tr.backward(lt)
    assert abs(float(lt) - loss_ref) <= TOL * abs(loss_ref)
    _compare(m, ref, "periodic ET force-loss")


@pytest.mark.parametrize("static_shapes", [False, True])
def test_tensornet_periodic_box_vs_oracle(static_shapes, large_switches):
    """TensorNet (128 ch, 2 layers, 32 RBF, cutoff 4.5) on a 1500-atom periodic water box: cell list,
    Morton renumbering (static_shapes off) or the reference CUDA padding semantics (on) vs the oracle."""
    from torchmdnet.models.model import create_model
    args = yaml_args("tensornet", embedding_dimension=128, num_layers=2, num_rbf=32, cutoff_upper=4.5,
                     max_num_neighbors=64, derivative=True, static_shapes=static_shapes)
    torch.manual_seed(0)
    m = create_model(args)
    # create_model does not forward static_shapes (neither does the reference's, models/model.py:81-84: TensorNet
    # keeps its default True); set it on the module as a user would
    m.representation_model.static_shapes = static_shapes
    m.representation_model.distance.resize_to_fit = not static_shapes
    z, pos, batch, L = _water_box(1500, seed=3)
    y_ref, f_ref = O.energy_forces(m.state_dict(), _cfg(args, L), z, pos, batch, static_shapes=static_shapes)
    m = _periodic(m.to(DEV), L)
    y, f = m(z.to(DEV), pos.float().to(DEV), batch.to(DEV))
    assert _rel(y, y_ref) < TOL, _rel(y, y_ref)
    assert _rel(f, f_ref) < TOL, _rel(f, f_ref)


# ----------------------------------------------------------------------------- reference-run periodic fixtures
@pytest.mark.parametrize("strategy", ["brute", "shared"])
@pytest.mark.parametrize("name", ["et_tiny_periodic_f64", "tn_tiny_periodic_static_f64", "tn_tiny_periodic_dyn_f64"])
@pytest.mark.parametrize("precision", [64, 32])
def test_periodic_model_matches_reference_fixture(name, strategy, precision):
    """Periodic MODEL parity against the reference itself (VERDICT r4 weak #1 / next #3b; before, periodic
    parity was pinned only by composition): ET-tiny and TensorNet-tiny (static padded and dynamic
    shapes) on a 120-atom rectangular water box, run by the reference (tests/golden/gen_reference_fixtures.py
    gen_periodic) -- energies and forces (fp64 1e-9, fp32 1e-4 relative) and, in fp64, the force-loss
    parameter gradients of the reference LNNP objective (double backward, 1e-7)."""
    from conftest import golden, state_dict_from
    from torchmdnet.models.model import create_model
    d = golden(name + ".npz")
    dtype = torch.float64 if precision == 64 else torch.float32
    if name.startswith("et"):
        args = yaml_args("equivariant-transformer", embedding_dimension=32, num_layers=2, num_rbf=16, num_heads=4,
                         max_num_neighbors=64, derivative=True, output_model="Scalar", precision=precision)
    else:
        args = yaml_args("tensornet", embedding_dimension=32, num_layers=2, num_rbf=16, max_num_neighbors=64,
                         cutoff_upper=4.5, derivative=True, output_model="Scalar", precision=precision)
    m = create_model(args)
    m.load_state_dict({k: torch.as_tensor(v) for k, v in state_dict_from(d).items()})
    if name.startswith("tn"):
        static = "static" in name
        m.representation_model.static_shapes = static
        m.representation_model.distance.resize_to_fit = not static
    m = m.to(DEV)
    dist = m.representation_model.distance
    dist.box = torch.as_tensor(d["box"]).to(dtype)
    dist.use_periodic = True
    dist.strategy = strategy
    z = torch.as_tensor(d["z"]).to(DEV)
    pos = torch.as_tensor(d["pos"]).to(dtype).to(DEV)
    batch = torch.as_tensor(d["batch"]).to(DEV)
    y, f = m(z, pos, batch)
    tol = 1e-9 if precision == 64 else TOL
    assert _rel(y, torch.as_tensor(d["y"])) < tol
    assert _rel(f, torch.as_tensor(d["neg_dy"])) < tol
    if precision == 64:
        loss = (y ** 2).sum() + (f ** 2).sum()
        names = [k for k in d.files if k.startswith("g2/")]
        params = dict(m.named_parameters())
        grads = torch.autograd.grad(loss, [params[k[3:]] for k in names], allow_unused=True)
        for k, g in zip(names, grads):
            ref = torch.as_tensor(d[k])
            if g is None:
                assert float(ref.abs().max()) == 0.0, k
                continue
            err = float((g.detach().cpu() - ref).norm() / ref.norm().clamp_min(1e-30))
            assert err < 1e-7 or float((g.detach().cpu() - ref).abs().max()) < 1e-10, (k, err)
