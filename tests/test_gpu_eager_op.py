"""Eval-mode eager evaluation through the C++ ``tmdnet::et_stack`` operator (torchmd_et.CPP_EAGER): the same
energies and forces as the Python layer stack, the same gradients to the parameters through the force
loss (the operator is differentiable to any order), and the route is really taken."""
import pytest
import torch

from conftest import yaml_args

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return float((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30))


def _args(H=128, L=4, R=32):
    return yaml_args("equivariant-transformer", embedding_dimension=H, num_layers=L, num_rbf=R, num_heads=8,
                     derivative=True)


def _model(H=128, L=4, R=32):
    from torchmdnet.models.model import create_model
    torch.manual_seed(0)
    return create_model(_args(H, L, R)).to(DEV)


@pytest.mark.parametrize("H,L,R", [(128, 4, 32), (64, 2, 32)])
def test_eval_eager_stack_operator_matches_python_stack(H, L, R, monkeypatch):
    from oracle import model_oracle as O
    from torchmdnet.models import torchmd_et
    m = _model(H, L, R).eval()
    z, pos, batch = O.qm9_like(16)
    y_ref, f_ref = O.energy_forces({k: v.cpu() for k, v in m.state_dict().items()}, dict(_args(H, L, R)), z, pos,
                                   batch)
    z, pos, batch = z.to(DEV), pos.float().to(DEV), batch.to(DEV)
    calls = []
    orig = torchmd_et.TorchMD_ET._stack_op
    monkeypatch.setattr(torchmd_et.TorchMD_ET, "_stack_op", lambda *a, **k: (calls.append(1), orig(*a, **k))[1])

    def run(cpp):
        monkeypatch.setattr(torchmd_et, "CPP_EAGER", cpp)
        y, f = m(z, pos, batch)
        return y.detach(), f.detach()

    y1, f1 = run(True)
    assert len(calls) == 1
    y0, f0 = run(False)
    assert len(calls) == 1
    assert _rel(y1.cpu(), y_ref.detach()) < 1e-5 and _rel(f1.cpu(), f_ref) < 1e-4
    assert _rel(y0.cpu(), y_ref.detach()) < 1e-5 and _rel(f0.cpu(), f_ref) < 1e-4
    assert _rel(y1, y0) < 1e-6 and _rel(f1, f0) < 1e-6


def test_eval_eager_stack_operator_parameter_gradients(monkeypatch):
    """Eval mode, energy differentiated to the parameters (no force loss): the operator's recompute
    backward against the Python stack's."""
    from oracle import model_oracle as O
    from torchmdnet.models import torchmd_et
    m = _model().eval()
    z, pos, batch = O.qm9_like(8)
    z, pos, batch = z.to(DEV), pos.float().to(DEV), batch.to(DEV)

    def grads(cpp):
        monkeypatch.setattr(torchmd_et, "CPP_EAGER", cpp)
        m.zero_grad(set_to_none=True)
        y, _ = m(z, pos.clone(), batch)
        y.sum().backward()
        return {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}

    a, b = grads(True), grads(False)
    assert a.keys() == b.keys() and len(a) > 0
    for n in a:
        assert _rel(a[n], b[n]) < 1e-4, n


def _stale_check(monkeypatch, mutate, scripted=False):
    """Evaluate through the C++ operator, rewrite the weights with ``mutate`` (no invalidation call of any
    kind), evaluate again: the result must be the Python stack's on the NEW weights."""
    from oracle import model_oracle as O
    from torchmdnet.models import torchmd_et
    m = _model(64, 2, 32).eval()
    z, pos, batch = O.qm9_like(8)
    z, pos, batch = z.to(DEV), pos.float().to(DEV), batch.to(DEV)
    monkeypatch.setattr(torchmd_et, "CPP_EAGER", True)
    run = torch.jit.script(m) if scripted else m
    y_old, _ = run(z, pos, batch)
    mutate(m)
    y1, f1 = run(z, pos, batch)
    monkeypatch.setattr(torchmd_et, "CPP_EAGER", False)
    y0, f0 = m(z, pos, batch)
    assert _rel(y_old.detach(), y0.detach()) > 1e-4  # (the premise: the weights did change the energy)
    assert _rel(y1.detach(), y0.detach()) < 1e-6 and _rel(f1.detach(), f0.detach()) < 1e-6


def _fused_adamw(m):
    params = [p for p in m.parameters() if p.requires_grad]
    vers = [p._version for p in params]
    for p in params:
        p.grad = torch.randn_like(p) * 0.1
    torch.optim.AdamW(params, lr=1e-2, fused=True).step()
    assert [p._version for p in params] == vers  # (the premise: a fused step bumps no version counter)


def _data_copy(m):
    g = torch.Generator(device=DEV).manual_seed(3)
    for name, p in m.named_parameters():
        if "attention_layers" in name:  # an EMA-style swap: p.data written, version counter untouched
            p.data.copy_(p.data + 0.05 * torch.randn(p.shape, device=DEV, generator=g))


@pytest.mark.parametrize("mutate", [_fused_adamw, _data_copy], ids=["fused_adamw", "data_copy"])
def test_cpp_route_sees_weight_updates_without_invalidation(mutate, monkeypatch):
    """a plain ``torch.optim.AdamW(fused=True)`` step, or ``p.data.copy_``, then an eval-mode
    evaluation through the C++ operator -- WITHOUT any cache invalidation call -- matches the Python stack on
    the new weights (the operator holds no packed copy: pack_stack takes views of the parameters)."""
    _stale_check(monkeypatch, mutate)


@pytest.mark.parametrize("mutate", [_fused_adamw, _data_copy], ids=["fused_adamw", "data_copy"])
def test_scripted_fused_eval_sees_weight_updates(mutate, monkeypatch):
    """The same through torch.jit.script(model.eval()) (one tmdnet::et_energy_forces operator)."""
    _stale_check(monkeypatch, mutate, scripted=True)
