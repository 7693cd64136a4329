"""TorchScript / dispatcher boundary (GPU): ``libtmdnet_torch.so`` registers the reference's
``torchmdnet_neighbors::get_neighbor_pairs`` and the ``tmdnet::*`` model-path operators with
TORCH_LIBRARY, so ``torch.jit.script`` sees them.

Ports of reference tests/test_neighbors.py:470-546 (test_jit_script_compatible) and
tests/test_model.py:42-84 (test_torchscript / test_torchscript_dynamic_shapes: energy, forces and a
second derivative of the scripted model), plus: scripted == eager model (fp32 1e-4 relative, the
north_star bar; fp64 against the oracle 1e-9), force-matching parameter gradients through the
scripted model, a jit.save / jit.load round trip, and the raw op's backward against the reference's
index_add expression to the second order (gradcheck / gradgradcheck in fp64).
"""
import io

import numpy as np
import pytest
import torch

from conftest import yaml_args
from oracle import model_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-12))


def _torch_lib_loaded():
    from torchmdnet import _native
    _native.load_torch_ops()
    maps = open("/proc/self/maps").read()
    assert "libtmdnet_torch.so" in maps and "libtmdnet_hip" in maps


# ----------------------------------------------------------------------------- raw neighbour op
GRID = [(s, nb, loop, tr, bt) for s in ("brute", "shared", "cell") for nb in (1, 128) for loop in (True, False)
        for tr in (True, False) for bt in (None, "triclinic", "rectangular")
        if not (bt == "triclinic" and s == "cell")]


@pytest.mark.parametrize("strategy,n_batches,loop,include_transpose,box_type", GRID)
def test_jit_script_compatible(strategy, n_batches, loop, include_transpose, box_type):
    """Reference test_neighbors.py:470-530: a scripted OptimizedDistance returns the reference pairs."""
    from torchmdnet.models.utils import OptimizedDistance
    _torch_lib_loaded()
    torch.manual_seed(4321)
    n_per = torch.randint(3, 100, size=(n_batches,))
    batch = torch.repeat_interleave(torch.arange(n_batches, dtype=torch.int64), n_per).to(DEV)
    lbox, cutoff = 10.0, 1.0
    pos = torch.rand(int(n_per.sum()), 3, device=DEV) * lbox
    pos[0, :] = 0.0
    pos[1, :] = 0.0
    pos.requires_grad_(True)
    box = None if box_type is None else torch.tensor([[lbox, 0.0, 0.0], [0.0, lbox, 0.0], [0.0, 0.0, lbox]]).to(DEV)
    rnb, rdl, rd = O.neighbors(pos.detach().cpu().double().numpy(), batch.cpu().numpy(), 0.0, cutoff, loop=loop,
                               include_transpose=include_transpose,
                               box=None if box is None else box.cpu().double().numpy(), sq_compare=True)
    rnb, rdl, rd = O.sort_pairs(rnb, rdl, rd)
    nl = torch.jit.script(OptimizedDistance(cutoff_lower=0.0, loop=loop, cutoff_upper=cutoff,
                                            max_num_pairs=rnb.shape[1], strategy=strategy, box=box,
                                            return_vecs=True, include_transpose=include_transpose))
    neighbors, distances, vecs = nl(pos, batch)
    nb, dl, d = O.sort_pairs(neighbors.cpu().numpy(), vecs.detach().cpu().numpy(), distances.detach().cpu().numpy())
    assert nb.shape == rnb.shape
    assert np.array_equal(nb, rnb)
    assert np.allclose(d, rd, atol=1e-5) and np.allclose(dl, rdl, atol=1e-5)


def _ref_backward(nb, dl, dist, gd, gr, n):
    """The reference's NeighborAutograd::backward (neighbors_cuda.cu:43-71) in plain torch."""
    zero = dist == 0
    g = gd.masked_fill(zero.unsqueeze(-1), 0) + dl / dist.masked_fill(zero, 1).unsqueeze(-1) * \
        gr.masked_fill(zero, 0).unsqueeze(-1)
    ei = nb.long().masked_fill(zero.unsqueeze(0), n)
    ei = ei.masked_fill(ei < 0, n)
    out = torch.zeros((n + 1, 3), dtype=dl.dtype, device=dl.device)
    return out.index_add(0, ei[0], g).index_add(0, ei[1], -g)[:n]


@pytest.mark.parametrize("include_transpose", [True, False])
def test_raw_op_backward_matches_reference_expression(include_transpose):
    from torchmdnet.neighbors import get_neighbor_pairs_kernel as op
    _torch_lib_loaded()
    torch.manual_seed(7)
    n = 300
    pos = (torch.rand(n, 3, device=DEV, dtype=torch.float64) * 6).requires_grad_(True)
    batch = torch.zeros(n, dtype=torch.long, device=DEV)
    nb, dl, d, num = op("brute", pos, batch, torch.empty(0, 0), False, 0.0, 2.0, 40000, True, include_transpose)
    assert int(num) < 40000
    gd = torch.randn_like(dl)
    gr = torch.randn_like(d)
    gpos, = torch.autograd.grad([dl, d], [pos], [gd, gr])
    ref = _ref_backward(nb, dl.detach(), d.detach(), gd, gr, n)
    assert _rel(gpos, ref) < 1e-12


def test_raw_op_gradgradcheck():
    """Second (and first) order of the raw op, fp64 finite differences (the reference differentiates
    its index_add backward by autograd; here the backward is a HIP kernel whose own backward is
    written out)."""
    from torchmdnet.neighbors import get_neighbor_pairs_kernel as op
    _torch_lib_loaded()
    torch.manual_seed(11)
    n = 24
    pos = (torch.rand(n, 3, device=DEV, dtype=torch.float64) * 3).requires_grad_(True)
    batch = torch.zeros(n, dtype=torch.long, device=DEV)
    box = torch.empty(0, 0)

    def f(p):
        nb, dl, d, num = op("brute", p, batch, box, False, 0.0, 1.5, 1000, True, True)
        return dl, d

    # the first-order kernel accumulates with atomics (as the reference's index_add_): fp64 sums in a
    # varying order, hence a round-off-sized reentrancy tolerance
    assert torch.autograd.gradcheck(f, (pos,), eps=1e-6, atol=1e-7, nondet_tol=1e-12)
    assert torch.autograd.gradgradcheck(f, (pos,), eps=1e-6, atol=1e-7, nondet_tol=1e-12)


# ----------------------------------------------------------------------------- scripted model
def _et_model(channels=128, layers=8, prior=None, dtype=torch.float32):
    from torchmdnet.models.model import create_model
    args = yaml_args("equivariant-transformer")
    if prior:
        args.update(prior_args={"max_z": 100})
    args.update(prior_model=prior, embedding_dimension=channels, num_layers=layers, derivative=True,
                precision=64 if dtype == torch.float64 else 32)
    torch.manual_seed(0)
    return create_model(args), args


def _batch(n_mol=8, dtype=torch.float32, seed=3):
    z, pos, batch = O.qm9_like(n_mol, seed)
    return z.to(DEV), pos.to(dtype).to(DEV), batch.to(DEV)


def test_torchscript_et_matches_eager_fp32():
    _torch_lib_loaded()
    model, _ = _et_model()
    model = model.to(DEV)
    scripted = torch.jit.script(model)
    z, pos, batch = _batch()
    y_e, f_e = model(z, pos.clone(), batch)
    y_s, f_s = scripted(z, pos.clone(), batch)
    assert _rel(y_s, y_e) < 1e-4
    assert _rel(f_s, f_e) < 1e-4


def test_torchscript_et_fp64_matches_oracle():
    _torch_lib_loaded()
    model, args = _et_model(channels=64, layers=3, dtype=torch.float64)
    z, pos, batch = O.qm9_like(4, 5)
    y_ref, f_ref = O.energy_forces(model.state_dict(), dict(args), z, pos, batch)
    scripted = torch.jit.script(model.to(DEV))
    y, f = scripted(z.to(DEV), pos.to(DEV), batch.to(DEV))
    assert _rel(y, y_ref) < 1e-9
    assert _rel(f, f_ref) < 1e-9


def test_torchscript_second_derivative():
    """Reference test_model.py:42-62: d(neg_dy)/d pos through the scripted model, against eager."""
    _torch_lib_loaded()
    model, _ = _et_model(channels=64, layers=3)
    model = model.to(DEV)
    scripted = torch.jit.script(model)
    z, pos, batch = _batch(4)
    outs = []
    for m in (model, scripted):
        p = pos.clone().requires_grad_(True)
        y, neg_dy = m(z, p, batch)
        ddy, = torch.autograd.grad([neg_dy], [p], grad_outputs=[torch.ones_like(neg_dy)])
        outs.append(ddy)
    assert _rel(outs[1], outs[0]) < 1e-4


def test_torchscript_dynamic_shapes():
    """Reference test_model.py:64-84: one scripted model, five different batch layouts."""
    _torch_lib_loaded()
    model, _ = _et_model(channels=64, layers=3)
    scripted = torch.jit.script(model.to(DEV))
    z, pos, batch = O.qm9_like(3, 9)
    for rep in range(5):
        zi = z.repeat_interleave(rep + 1).to(DEV)
        pi = pos.float().repeat_interleave(rep + 1, dim=0).to(DEV)
        pi = pi + 0.05 * torch.randn_like(pi)
        bi = torch.randint(0, 10, (zi.shape[0],)).sort()[0].to(DEV)
        pi.requires_grad_(True)
        y, neg_dy = scripted(zi, pi, bi)
        ddy, = torch.autograd.grad([neg_dy], [pi], grad_outputs=[torch.ones_like(neg_dy)])
        assert torch.isfinite(y).all() and torch.isfinite(neg_dy).all() and torch.isfinite(ddy).all()
        y_e, f_e = model(zi, pi.detach().clone(), bi)
        assert _rel(y, y_e) < 1e-4 and _rel(neg_dy, f_e) < 1e-4


def test_torchscript_force_matching_gradients():
    """Training through the scripted model (energy + force loss, parameter gradients by double
    backward) equals the eager model's."""
    _torch_lib_loaded()
    model, _ = _et_model(channels=64, layers=2, prior="Atomref")
    with torch.no_grad():  # non-zero per-element offsets
        model.prior_model[0].atomref.weight.uniform_(-1, 1)
    model = model.to(DEV)
    scripted = torch.jit.script(model)
    z, pos, batch = _batch(6)
    torch.manual_seed(1)
    y_t = torch.randn(6, 1, device=DEV)
    f_t = torch.randn_like(pos)
    grads = []
    for m in (model, scripted):
        named = [(n, p) for n, p in m.named_parameters() if p.requires_grad]
        y, neg_dy = m(z, pos.clone(), batch)
        loss = ((y - y_t) ** 2).mean() + ((neg_dy - f_t) ** 2).mean()
        grads.append(torch.autograd.grad(loss, [p for _, p in named], allow_unused=True))
    names = [n for n, _ in named]
    n_checked = 0
    for name, ge, gs in zip(names, *grads):
        if ge is None:
            assert gs is None or gs.abs().max() == 0, name
            continue
        assert gs is not None, name
        assert _rel(gs, ge) < 2e-4, name
        n_checked += 1
    assert n_checked > 20


def test_torchscript_save_load_roundtrip():
    _torch_lib_loaded()
    model, _ = _et_model(channels=64, layers=2)
    scripted = torch.jit.script(model.to(DEV))
    buf = io.BytesIO()
    torch.jit.save(scripted, buf)
    buf.seek(0)
    loaded = torch.jit.load(buf, map_location=DEV)
    z, pos, batch = _batch(4)
    y0, f0 = scripted(z, pos.clone(), batch)
    y1, f1 = loaded(z, pos.clone(), batch)
    assert torch.equal(y0, y1) and torch.equal(f0, f1)
    assert set(loaded.state_dict()) == set(model.state_dict())


# ----------------------------------------------------------------------------- scripted TensorNet
def _tn_model(group="O(3)", static_shapes=True, dtype=torch.float32):
    from torchmdnet.models.model import create_model
    args = yaml_args("tensornet", derivative=True, equivariance_invariance_group=group,
                     precision=64 if dtype == torch.float64 else 32)
    torch.manual_seed(0)
    m = create_model(args)
    m.representation_model.static_shapes = static_shapes  # (create_model does not take it, as the reference)
    return m, args


@pytest.mark.parametrize("group", ["O(3)", "SO(3)"])
def test_torchscript_tensornet_matches_eager(group):
    """Reference test_model.py:42-62 for TensorNet (static_shapes, the reference default): energy,
    forces and the second derivative of the scripted model equal the eager HIP path."""
    _torch_lib_loaded()
    model, _ = _tn_model(group)
    model = model.to(DEV)
    scripted = torch.jit.script(model)
    z, pos, batch = _batch(6)
    res = []
    for m in (model, scripted):
        p = pos.clone().requires_grad_(True)
        y, neg_dy = m(z, p, batch)
        ddy, = torch.autograd.grad([neg_dy], [p], grad_outputs=[torch.ones_like(neg_dy)])
        res.append((y, neg_dy, ddy))
    for a, b in zip(res[1], res[0]):
        assert _rel(a, b) < 1e-4


@pytest.mark.parametrize("family", ["et", "tensornet"])
def test_torchscript_after_eager_runs(family):
    """A model that already ran eagerly (host-side scratch: force seeds, stacked projection rows) still
    scripts, in train and eval mode, and matches the eager outputs (the order the bench uses)."""
    _torch_lib_loaded()
    model = (_et_model()[0] if family == "et" else _tn_model("O(3)")[0]).to(DEV)
    z, pos, batch = _batch()
    y_e, f_e = model(z, pos.clone(), batch)
    for train in (True, False):
        model.train(train)
        y_s, f_s = torch.jit.script(model)(z, pos.clone(), batch)
        assert _rel(y_s, y_e) < 1e-4 and _rel(f_s, f_e) < 1e-4


@pytest.mark.parametrize("static_shapes", [True, False])
def test_torchscript_tensornet_fp64_matches_oracle(static_shapes):
    _torch_lib_loaded()
    model, args = _tn_model(dtype=torch.float64, static_shapes=static_shapes)
    z, pos, batch = O.qm9_like(3, 4)
    y_ref, f_ref = O.energy_forces(model.state_dict(), dict(args), z, pos, batch, static_shapes=static_shapes)
    scripted = torch.jit.script(model.to(DEV))
    y, f = scripted(z.to(DEV), pos.to(DEV), batch.to(DEV))
    assert _rel(y, y_ref) < 1e-9
    assert _rel(f, f_ref) < 1e-9


def test_torchscript_tensornet_force_matching_gradients():
    _torch_lib_loaded()
    model, _ = _tn_model("O(3)")
    model = model.to(DEV)
    scripted = torch.jit.script(model)
    z, pos, batch = _batch(4)
    torch.manual_seed(2)
    y_t, f_t = torch.randn(4, 1, device=DEV), torch.randn_like(pos)
    grads = []
    for m in (model, scripted):
        params = [p for p in m.parameters() if p.requires_grad]
        y, neg_dy = m(z, pos.clone(), batch)
        loss = ((y - y_t) ** 2).mean() + ((neg_dy - f_t) ** 2).mean()
        grads.append(torch.autograd.grad(loss, params, allow_unused=True))
    for ge, gs in zip(*grads):
        if ge is not None:
            assert _rel(gs, ge) < 2e-4


# ----------------------------------------------------------------------------- the fused scripted stack
def test_torchscript_et_runs_fused_stack_operator():
    """The scripted ET model runs its interaction layers as ONE tmdnet::et_stack operator (the eager
    stack's fused launches), not the per-layer ATen loop."""
    _torch_lib_loaded()
    model, _ = _et_model(channels=64, layers=2)
    scripted = torch.jit.script(model.to(DEV))
    # (forward calls _forward_script: the inlined graph holds every method it reaches)
    graph = str(scripted.representation_model.forward.inlined_graph)
    assert "tmdnet::et_stack" in graph


@pytest.mark.parametrize("influence", ["keys", "values", "none"])
def test_torchscript_fused_stack_distance_influence(influence):
    """tmdnet::et_stack with dk only, dv only and no distance projection: energies, forces and the
    second derivative equal the eager model's."""
    _torch_lib_loaded()
    from torchmdnet.models.model import create_model
    args = yaml_args("equivariant-transformer")
    args.update(embedding_dimension=64, num_layers=3, derivative=True, distance_influence=influence)
    torch.manual_seed(0)
    model = create_model(args).to(DEV)
    scripted = torch.jit.script(model)
    z, pos, batch = _batch(4)
    outs = []
    for m in (model, scripted):
        p = pos.clone().requires_grad_(True)
        y, neg_dy = m(z, p, batch)
        ddy, = torch.autograd.grad([neg_dy], [p], grad_outputs=[torch.ones_like(neg_dy)])
        outs.append((y.detach(), neg_dy.detach(), ddy))
    for a, b in zip(outs[1], outs[0]):
        assert _rel(a, b) < 1e-4


def test_torchscript_fused_stack_no_stale_pack_across_models():
    """et_stack caches its packed weights per parameter set.  Two models built and loaded the same way
    (identical version counters) must not share a pack even when the second model's parameters land at
    the first one's freed addresses (the key holds weak references to the storages)."""
    _torch_lib_loaded()
    import gc
    from torchmdnet.models.model import create_model
    args = yaml_args("equivariant-transformer")
    args.update(embedding_dimension=64, num_layers=2, derivative=True)
    z, pos, batch = _batch(4)
    for seed in (0, 1, 2):
        torch.manual_seed(seed)
        model = create_model(args).to(DEV)
        scripted = torch.jit.script(model)
        y_s, f_s = scripted(z, pos.clone(), batch)
        y_e, f_e = model(z, pos.clone(), batch)
        assert _rel(y_s, y_e) < 1e-4 and _rel(f_s, f_e) < 1e-4, seed
        del model, scripted, y_s, f_s, y_e, f_e
        gc.collect()
    # in-place writes that bypass the version counter need the explicit invalidation
    torch.manual_seed(3)
    model = create_model(args).to(DEV)
    scripted = torch.jit.script(model)
    scripted(z, pos.clone(), batch)
    with torch.no_grad():
        for p in model.parameters():
            p.data.mul_(0.5)
    torch.ops.tmdnet.et_stack_invalidate()
    y_s, f_s = scripted(z, pos.clone(), batch)
    y_e, f_e = model(z, pos.clone(), batch)
    assert _rel(y_s, y_e) < 1e-4 and _rel(f_s, f_e) < 1e-4


@pytest.mark.parametrize("neighbor_embedding", [True, False])
def test_torchscript_fused_eval_matches_eager_and_oracle(neighbor_embedding):
    """Eval-mode TorchScript (the MD-engine form, reference README.md:6) runs the whole energy + force
    evaluation as ONE operator, tmdnet::et_energy_forces: equal to the eager model and to the fp64 oracle
    (fp32 bar 1e-4); in train mode the scripted model keeps the differentiable operator path."""
    from torchmdnet.models.model import create_model
    _torch_lib_loaded()
    args = yaml_args("equivariant-transformer")
    args.update(prior_model=None, embedding_dimension=128, num_layers=8, derivative=True,
                neighbor_embedding=neighbor_embedding)
    torch.manual_seed(0)
    model = create_model(args).to(DEV).eval()
    assert model.fused_eval
    scripted = torch.jit.script(model)
    assert "et_energy_forces" in str(scripted.inlined_graph)
    z, pos, batch = _batch(8)
    y_e, f_e = model(z, pos.clone(), batch)
    y_s, f_s = scripted(z, pos.clone(), batch)
    assert _rel(y_s, y_e) < 1e-4 and _rel(f_s, f_e) < 1e-4
    y_ref, f_ref = O.energy_forces(model.state_dict(), dict(args), z.cpu(), pos.cpu().double(), batch.cpu())
    assert _rel(y_s, y_ref) < 1e-4 and _rel(f_s, f_ref) < 1e-4
    scripted.train()
    p = pos.clone().requires_grad_(True)
    y_t, f_t = scripted(z, p, batch)
    assert f_t.requires_grad and _rel(f_t, f_e) < 1e-4


def test_torchscript_fused_eval_periodic_cell_list():
    """The fused evaluation on a periodic box with the cell list (its neighbour build and minimum-image
    geometry inside the operator) against the eager model."""
    from torchmdnet.models.model import create_model
    _torch_lib_loaded()
    args = yaml_args("equivariant-transformer")
    args.update(prior_model=None, embedding_dimension=128, num_layers=3, derivative=True, max_num_neighbors=128)
    torch.manual_seed(0)
    model = create_model(args).to(DEV).eval()
    n = 600
    g = torch.Generator().manual_seed(2)
    L = (n / 0.1003) ** (1.0 / 3.0)
    pos = (torch.rand(n, 3, generator=g, dtype=torch.float64) * L).float().to(DEV)
    z = torch.tensor([8, 1, 1], dtype=torch.long).repeat(n // 3 + 1)[:n].to(DEV)
    batch = torch.zeros(n, dtype=torch.long, device=DEV)
    d = model.representation_model.distance
    d.box = torch.eye(3) * L
    d.use_periodic = True
    d.strategy = "cell"
    scripted = torch.jit.script(model)
    y_e, f_e = model(z, pos.clone(), batch)
    y_s, f_s = scripted(z, pos.clone(), batch)
    assert _rel(y_s, y_e) < 1e-4 and _rel(f_s, f_e) < 1e-4


@pytest.mark.parametrize("strategy", ["cell", "brute"])
def test_torchscript_fused_eval_large_system_forms(monkeypatch, strategy):
    """The MD-engine form at C5 layout: tmdnet::et_energy_forces with its large-system
    switches forced on a 3000-atom periodic water box -- Morton renumbering, pair-shared rows
    (tmdnet_pair_index), planar v rows and the fused-projection layer kernels, node mixes above 16k rows
    on tmdnet_gemm_x3_f32 -- against the eager model with the same switches forced (1e-4), and against
    the eager model on its default small-system path; forces come back in the caller's atom order."""
    from torchmdnet import et_stack, kernels
    from torchmdnet.models.model import create_model
    _torch_lib_loaded()
    args = yaml_args("equivariant-transformer")
    args.update(prior_model=None, embedding_dimension=128, num_layers=4, derivative=True, max_num_neighbors=128)
    torch.manual_seed(0)
    model = create_model(args).to(DEV).eval()
    n = 3000
    g = torch.Generator().manual_seed(5)
    L = (n / 0.1003) ** (1.0 / 3.0)
    pos = (torch.rand(n, 3, generator=g, dtype=torch.float64) * L).float().to(DEV)
    z = torch.tensor([8, 1, 1], dtype=torch.long).repeat(n // 3 + 1)[:n].to(DEV)
    batch = torch.zeros(n, dtype=torch.long, device=DEV)
    d = model.representation_model.distance
    d.box = torch.eye(3) * L
    d.use_periodic = True
    d.strategy = strategy
    y_plain, f_plain = model(z, pos.clone(), batch)  # eager, small-system forms
    monkeypatch.setattr(kernels, "REORDER_MIN_ATOMS", 0)
    monkeypatch.setattr(et_stack, "PLANAR_MIN_EDGES", 0)
    monkeypatch.setattr(et_stack, "FEP_MIN_EDGES", 0)
    fused_calls = []
    orig = kernels.et_fused_fwd_launch
    monkeypatch.setattr(kernels, "et_fused_fwd_launch", lambda *a, **k: fused_calls.append(1) or orig(*a, **k))
    y_e, f_e = model(z, pos.clone(), batch)
    assert len(fused_calls) == 4
    scripted = torch.jit.script(model)
    prev = torch.ops.tmdnet.set_large_system_thresholds(0, 0)
    try:
        y_s, f_s = scripted(z, pos.clone(), batch)
    finally:
        torch.ops.tmdnet.set_large_system_thresholds(prev[0], prev[1])
    assert not f_s.requires_grad
    assert _rel(y_s, y_e) < 1e-4 and _rel(f_s, f_e) < 1e-4
    assert _rel(y_s, y_plain) < 1e-4 and _rel(f_s, f_plain) < 1e-4
