"""No library GEMM on the timed configurations: every ATen matrix product (mm, addmm, bmm,
baddbmm, mv, addmv -- what torch.mm / F.linear / @ / autograd's own backward formulas dispatch to, i.e. hipBLASLt /
rocBLAS ``Cijk_*`` launches) is recorded by a TorchDispatchMode while the bench workloads run once eagerly:
C2 (ET-QM9 energy + forces, the graph-captured bench step's code), the ET-QM9 training step (E + F loss, the
double backward, AdamW), TensorNet C3 (inference and training) and both C5 arms at full size (50,001-atom water
box, ET and TensorNet).  The hand GEMMs (tmdnet_gemm_*, k_gemm_x3, the TN weight gradients) are not ATen ops."""
import os
import sys

import pytest
import torch
from torch.utils._python_dispatch import TorchDispatchMode

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
DEV = torch.device("cuda", 0)
aten = torch.ops.aten
_GEMMS = {aten.mm, aten.addmm, aten.bmm, aten.baddbmm, aten.mv, aten.addmv, aten._addmm_activation, aten.addbmm}


class _LibraryGemms(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.hits = []

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        if func.overloadpacket in _GEMMS:
            shapes = [tuple(a.shape) for a in args if isinstance(a, torch.Tensor)]
            self.hits.append(f"{func} {shapes}")
        return func(*args, **(kwargs or {}))


def _check(fn):
    with _LibraryGemms() as m:
        fn()
        torch.cuda.synchronize()
    assert not m.hits, m.hits[:10]


def test_c2_energy_forces_and_training_step():
    import bench
    from torchmdnet.models.model import create_model
    from torchmdnet.training import LNNPStep
    torch.manual_seed(0)
    model = create_model(bench.et_args(128)).to(DEV)
    z, pos, batch = bench.qm9_like(32, 1)
    z, pos, batch = z.to(DEV), pos.float().to(DEV), batch.to(DEV)
    model(z, pos, batch)  # (first call: lazily built state outside the recorded region)
    _check(lambda: model(z, pos, batch))
    model.eval()  # eval mode: the layer stack as the C++ tmdnet::et_stack operator
    model(z, pos, batch)
    _check(lambda: model(z, pos, batch))
    model.train()
    g = torch.Generator().manual_seed(100)
    y_lab, f_lab = torch.randn(32, 1, generator=g).to(DEV), torch.randn(z.shape[0], 3, generator=g).to(DEV)
    trainer = LNNPStep(model, lr=1e-4)
    trainer.step(z, pos, batch, y_lab, f_lab)
    _check(lambda: trainer.step(z, pos, batch, y_lab, f_lab))


def test_tensornet_c3_inference_and_training():
    import bench
    from torchmdnet.models.model import create_model
    from torchmdnet.training import LNNPStep
    torch.manual_seed(0)
    model = create_model(bench.tn_args()).to(DEV)
    z, pos, batch = bench.rmd17_like(8, 1)
    z, pos, batch = z.to(DEV), pos.float().to(DEV), batch.to(DEV)
    model(z, pos, batch)
    _check(lambda: model(z, pos, batch))
    g = torch.Generator().manual_seed(100)
    y_lab, f_lab = torch.randn(8, 1, generator=g).to(DEV), torch.randn(z.shape[0], 3, generator=g).to(DEV)
    trainer = LNNPStep(model, lr=1e-4)
    trainer.step(z, pos, batch, y_lab, f_lab)
    _check(lambda: trainer.step(z, pos, batch, y_lab, f_lab))


def test_c5_water_box_both_arms():
    import bench
    from torchmdnet.models.model import create_model
    n = 50001
    args = bench.et_args(128)
    args.update(max_num_neighbors=128)
    torch.manual_seed(0)
    model = create_model(args).to(DEV)
    d = model.representation_model.distance
    L = (n / 0.1003) ** (1.0 / 3.0)
    g = torch.Generator().manual_seed(7)
    pos = (torch.rand(n, 3, generator=g, dtype=torch.float64) * L).float().to(DEV)
    z = torch.tensor([8, 1, 1], dtype=torch.long).repeat(n // 3 + 1)[:n].to(DEV)
    batch = torch.zeros(n, dtype=torch.long, device=DEV)
    d.box = torch.eye(3, dtype=torch.float32) * L
    d.use_periodic = True
    d.strategy = "cell"
    model(z, pos, batch)
    _check(lambda: model(z, pos, batch))
    del model
    torch.cuda.empty_cache()
    model, z, pos, batch, _ = bench.tn_water_box_model(n, True, 0, DEV)
    model(z, pos, batch)
    _check(lambda: model(z, pos, batch))
