"""Runs N eager ET-QM9 energy+force steps (bench workload); used under rocprofv3 --kernel-trace to list
the kernel sequence of one step (tools/step_trace.py; see profiles/)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "torchmd-net_amd"), ROOT]
import torch  # noqa: E402

from bench import et_args, qm9_like  # noqa: E402
from torchmdnet.models.model import create_model  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = create_model(et_args(128)).to(dev)
z, pos, batch = qm9_like(32, 1)
z, pos, batch = z.to(dev), pos.float().to(dev), batch.to(dev)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
for _ in range(n):
    y, f = model(z, pos, batch)
torch.cuda.synchronize()
torch.cuda._sleep(100)  # marker kernels bracket the traced step
y, f = model(z, pos, batch)
torch.cuda._sleep(100)
torch.cuda.synchronize()
