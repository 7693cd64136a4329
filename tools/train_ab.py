"""Eager ET-QM9 training-step time, fused EquivariantScalar head vs the module-by-module head, same
box (diagnosis)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "torchmd-net_amd"), ROOT]
import torch  # noqa: E402
from bench import et_args, qm9_like  # noqa: E402
from torchmdnet.models.model import create_model  # noqa: E402
from torchmdnet.models.output_modules import EquivariantScalar  # noqa: E402
from torchmdnet.training import LNNPStep  # noqa: E402

dev = torch.device("cuda", 0)
fused = EquivariantScalar.pre_reduce


def unfused(self, x, v, z, pos, batch):
    for layer in self.output_network:
        x, v = layer(x, v)
    return x + v.sum() * 0


def run(tag):
    torch.manual_seed(0)
    model = create_model(et_args(128)).to(dev)
    z, pos, batch = qm9_like(32, gen_seed=1)
    g = torch.Generator().manual_seed(100)
    y = torch.randn(32, 1, generator=g).to(dev)
    f = torch.randn(z.shape[0], 3, generator=g).to(dev)
    z, pos, batch = z.to(dev), pos.float().to(dev), batch.to(dev)
    tr = LNNPStep(model, lr=4e-4)
    for _ in range(5):
        tr.step(z, pos, batch, y, f)
    torch.cuda.synchronize()
    t = time.perf_counter()
    n = 20
    for _ in range(n):
        tr.step(z, pos, batch, y, f)
    torch.cuda.synchronize()
    print(tag, f"{1000 * (time.perf_counter() - t) / n:.2f} ms/step", flush=True)


for rep in range(2):
    EquivariantScalar.pre_reduce = fused
    run("fused")
    EquivariantScalar.pre_reduce = unfused
    run("unfused")
