"""precision=16 (VERDICT r5 missing #3 / X1): the reference maps it to float16 (models/utils.py:586,
scripts/train.py:43).  Here the model STORES every floating parameter and buffer in float16 (the reference's
state_dict dtype) and the HIP path computes in float32 on upcasts of them (TorchMD_Net.half_storage_); energies
and forces come back in float16.  Gates (SURVEY §8(d) bf16/reduced-precision gate):
* against the fp64 oracle on the SAME fp16-rounded weights: energy and forces within 2e-3 relative (the fp16
  rounding of the outputs; the arithmetic is the fp32 path's);
* against the fp64 oracle on the ORIGINAL fp32 weights (what switching a model to precision 16 costs): energy
  within 2e-2 relative;
* rotation equivariance: energy invariant and forces co-rotating within 2e-3;
* a force-matching training step reaches the float16 parameters (gradients finite, same dtype)."""
import pytest
import torch

from conftest import yaml_args
from oracle import model_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _args(model, precision):
    if model == "et":
        return yaml_args("equivariant-transformer", embedding_dimension=128, num_layers=8, num_rbf=64, num_heads=8,
                         derivative=True, precision=precision)
    return yaml_args("tensornet", embedding_dimension=128, num_layers=2, num_rbf=32, cutoff_upper=4.5,
                     max_num_neighbors=64, derivative=True, precision=precision)


def _rot(seed):
    g = torch.Generator().manual_seed(seed)
    q, _ = torch.linalg.qr(torch.randn(3, 3, generator=g, dtype=torch.float64))
    if torch.det(q) < 0:
        q[:, 0] = -q[:, 0]
    return q


@pytest.mark.parametrize("model", ["et", "tn"])
def test_precision16_against_oracle_and_equivariance(model):
    from torchmdnet.models.model import create_model
    torch.manual_seed(0)
    m32 = create_model(_args(model, 32))
    torch.manual_seed(0)
    m16 = create_model(_args(model, 16))
    assert all(p.dtype == torch.float16 for p in m16.parameters())
    m16.load_state_dict({k: v.half() if v.is_floating_point() else v for k, v in m32.state_dict().items()})
    z, pos, batch = O.qm9_like(16)
    cfg = dict(_args(model, 32))
    sd16 = {k: v.double() if v.is_floating_point() else v for k, v in m16.state_dict().items()}
    y_ref16, f_ref16 = O.energy_forces(sd16, cfg, z, pos, batch)
    y_ref32, _ = O.energy_forces(m32.state_dict(), cfg, z, pos, batch)
    m16 = m16.to(DEV)
    y, f = m16(z.to(DEV), pos.float().to(DEV), batch.to(DEV))
    assert y.dtype == torch.float16 and f.dtype == torch.float16
    assert _rel(y, y_ref16) < 2e-3 and _rel(f, f_ref16) < 2e-3
    assert _rel(y, y_ref32) < 2e-2
    R = _rot(3).float().to(DEV)
    yr, fr = m16(z.to(DEV), (pos.float().to(DEV) @ R.t()), batch.to(DEV))
    assert _rel(yr, y) < 2e-3
    assert _rel(fr, f.float() @ R.t()) < 2e-3


def test_precision16_training_step_reaches_fp16_parameters():
    from torchmdnet.models.model import create_model
    torch.manual_seed(0)
    m = create_model(_args("et", 16)).to(DEV)
    z, pos, batch = O.qm9_like(8)
    z, pos, batch = z.to(DEV), pos.float().to(DEV), batch.to(DEV)
    y, f = m(z, pos, batch)
    loss = y.float().pow(2).mean() + f.float().pow(2).mean()
    loss.backward()
    grads = [p.grad for p in m.parameters() if p.requires_grad]
    assert all(g is not None and g.dtype == torch.float16 for g in grads)
    assert all(torch.isfinite(g.float()).all() for g in grads)
    assert sum(float(g.float().abs().sum()) for g in grads) > 0
