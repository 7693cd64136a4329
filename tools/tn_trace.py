"""Eager TensorNet-rMD17 (C3) energy+force steps bracketed by marker kernels, for rocprofv3 traces
(tools/trace_summary.py)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "torchmd-net_amd"), ROOT]
import torch  # noqa: E402
import yaml  # noqa: E402

from bench import rmd17_like  # noqa: E402
from torchmdnet.models.model import create_model  # noqa: E402

dev = torch.device("cuda", 0)
with open(os.path.join(ROOT, "tests", "golden", "configs", "tensornet_rmd17.yaml")) as f:
    args = yaml.safe_load(f)
args.update(prior_model=None, precision=32, derivative=True)
torch.manual_seed(0)
model = create_model(args).to(dev)
z, pos, batch = rmd17_like(8, 1)
z, pos, batch = z.to(dev), pos.float().to(dev), batch.to(dev)
for _ in range(3):
    model(z, pos, batch)
torch.cuda.synchronize()
torch.cuda._sleep(100)
y, f = model(z, pos, batch)
torch.cuda._sleep(100)
torch.cuda.synchronize()
