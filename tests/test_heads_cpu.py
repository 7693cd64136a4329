"""Secondary output heads and the Atomref prior on CPU (plain tensor code, no kernels): each head's
pre_reduce / post_reduce against the physical quantity it names, restated independently here.

Interfaces: reference torchmdnet/models/output_modules.py:117-207 (DipoleMoment, EquivariantDipoleMoment,
ElectronicSpatialExtent, EquivariantElectronicSpatialExtent, EquivariantVectorOutput) and
torchmdnet/priors/atomref.py:8-42 (Atomref).  Parity is pinned here against the definitions (dipole
= sum q_i (r_i - r_com), <R^2> = sum q_i |r_i - r_com|^2), not against reference-run fixtures: the reference
tests hold none for these heads ("parity unpinned" against the reference itself)."""
import warnings

import numpy as np
import pytest
import torch

from torchmdnet.models import output_modules as om
from torchmdnet.priors import Atomref
from torchmdnet.utils import atomic_masses


def _inputs(seed=0, H=16):
    g = torch.Generator().manual_seed(seed)
    z = torch.tensor([6, 1, 1, 8, 1, 7, 1, 1, 1], dtype=torch.long)
    pos = torch.randn(9, 3, generator=g, dtype=torch.float64)
    batch = torch.tensor([0, 0, 0, 1, 1, 2, 2, 2, 2])
    x = torch.randn(9, H, generator=g, dtype=torch.float64)
    v = torch.randn(9, 3, H, generator=g, dtype=torch.float64)
    return z, pos, batch, x, v


def _com_offsets(z, pos, batch):
    out = torch.empty_like(pos)
    m = torch.as_tensor(atomic_masses, dtype=pos.dtype)[z]
    for b in batch.unique():
        sel = batch == b
        c = (m[sel, None] * pos[sel]).sum(0) / m[sel].sum()
        out[sel] = pos[sel] - c
    return out


def _reduce(x, batch):
    return torch.stack([x[batch == b].sum(0) for b in batch.unique()])


def test_dipole_moment():
    z, pos, batch, x, v = _inputs()
    torch.manual_seed(0)
    head = om.DipoleMoment(16, dtype=torch.float64)
    q = head.output_network(x)
    want = (_reduce(q * _com_offsets(z, pos, batch), batch)).norm(dim=-1, keepdim=True)
    got = head.post_reduce(head.reduce(head.pre_reduce(x, v, z, pos, batch), batch))
    assert torch.allclose(got, want, rtol=1e-12, atol=1e-12)
    assert not head.allow_prior_model
    assert "atomic_mass" in head.state_dict()


def test_equivariant_dipole_moment():
    z, pos, batch, x, v = _inputs(1)
    torch.manual_seed(0)
    head = om.EquivariantDipoleMoment(16, dtype=torch.float64)
    xs, vs = x, v
    for blk in head.output_network:
        xs, vs = blk(xs, vs)
    per_atom = xs * _com_offsets(z, pos, batch) + vs[..., 0]
    want = _reduce(per_atom, batch).norm(dim=-1, keepdim=True)
    got = head.post_reduce(head.reduce(head.pre_reduce(x, v, z, pos, batch), batch))
    assert torch.allclose(got, want, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("cls", [om.ElectronicSpatialExtent, om.EquivariantElectronicSpatialExtent])
def test_electronic_spatial_extent(cls):
    z, pos, batch, x, v = _inputs(2)
    torch.manual_seed(0)
    head = cls(16, dtype=torch.float64)
    r2 = _com_offsets(z, pos, batch).pow(2).sum(1, keepdim=True)
    want = _reduce(head.output_network(x) * r2, batch)
    got = head.reduce(head.pre_reduce(x, v, z, pos, batch), batch)
    assert torch.allclose(got, want, rtol=1e-12, atol=1e-12)


def test_equivariant_vector_output_rotates_with_inputs():
    z, pos, batch, x, v = _inputs(3)
    torch.manual_seed(0)
    head = om.EquivariantVectorOutput(16, dtype=torch.float64)
    out = head.pre_reduce(x, v, z, pos, batch)
    assert out.shape == (9, 3)
    th = 0.7
    R = torch.tensor([[np.cos(th), -np.sin(th), 0], [np.sin(th), np.cos(th), 0], [0, 0, 1]], dtype=torch.float64)
    out_r = head.pre_reduce(x, torch.einsum("ij,njh->nih", R, v), z, pos @ R.T, batch)
    assert torch.allclose(out_r, out @ R.T, rtol=1e-10, atol=1e-12)


def test_seeded_parameters_follow_creation_order():
    """Same seed, same weights: the heads draw their initial weights in the reference's order (Linear
    construction, then xavier per layer)."""
    torch.manual_seed(5)
    a = om.ElectronicSpatialExtent(16)
    torch.manual_seed(5)
    ref0 = torch.nn.Linear(16, 8)
    ref1 = torch.nn.Linear(8, 1)
    torch.nn.init.xavier_uniform_(ref0.weight)
    torch.nn.init.xavier_uniform_(ref1.weight)
    assert torch.equal(a.output_network[0].weight, ref0.weight)
    assert torch.equal(a.output_network[2].weight, ref1.weight)


def test_atomref_table_and_errors():
    z = torch.tensor([1, 6, 8, 1])
    prior = Atomref(max_z=10)
    assert prior.initial_atomref.shape == (10, 1)
    assert torch.equal(prior.pre_reduce(torch.ones(4, 1), z, None, None, None), torch.ones(4, 1))
    with torch.no_grad():
        prior.atomref.weight[6] = 2.5
    assert float(prior.pre_reduce(torch.zeros(4, 1), z, None, None, None)[1]) == 2.5
    prior.reset_parameters()
    assert float(prior.atomref.weight.abs().sum()) == 0.0
    assert prior.get_init_args() == {"max_z": 10}
    assert set(prior.state_dict()) == {"initial_atomref", "atomref.weight"}
    with pytest.raises(ValueError):
        Atomref()

    class _DS:
        def __init__(self, t):
            self.t = t

        def get_atomref(self):
            return self.t

    p = Atomref(dataset=_DS(torch.arange(5, dtype=torch.float32)))
    assert p.initial_atomref.shape == (5, 1) and float(p.atomref.weight[3]) == 3.0
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        p = Atomref(dataset=_DS(None))
    assert p.initial_atomref.shape == (100, 1) and any("Atomref" in str(x.message) for x in w)
