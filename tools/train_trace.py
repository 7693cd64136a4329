"""Eager ET-QM9 training steps (bench workload) bracketed by marker kernels, for rocprofv3 traces."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "torchmd-net_amd"), ROOT]
import torch  # noqa: E402

from bench import et_args, qm9_like  # noqa: E402
from torchmdnet.models.model import create_model  # noqa: E402
from torchmdnet.training import LNNPStep  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = create_model(et_args(128)).to(dev)
z, pos, batch = qm9_like(32, 1)
z, pos, batch = z.to(dev), pos.float().to(dev), batch.to(dev)
y_lab = torch.randn(32, 1, device=dev)
f_lab = torch.randn(z.shape[0], 3, device=dev)
tr = LNNPStep(model, lr=4e-4)
for _ in range(3):
    tr.step(z, pos, batch, y_lab, f_lab)
torch.cuda.synchronize()
torch.cuda._sleep(100)
tr.step(z, pos, batch, y_lab, f_lab)
torch.cuda._sleep(100)
torch.cuda.synchronize()
