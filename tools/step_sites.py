"""Profile one eager ET-QM9 energy+force step (bench workload) with torch.profiler (CPU + GPU
activity, Python stacks) and write a chrome trace for tools/kernel_sites.py (diagnosis)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "torchmd-net_amd"), ROOT]
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from bench import et_args, qm9_like  # noqa: E402
from torchmdnet.models.model import create_model  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = create_model(et_args(128)).to(dev)
z, pos, batch = qm9_like(32, 1)
z, pos, batch = z.to(dev), pos.float().to(dev), batch.to(dev)
for _ in range(4):
    y, f = model(z, pos, batch)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True,
             record_shapes=True) as prof:
    y, f = model(z, pos, batch)
    torch.cuda.synchronize()
prof.export_chrome_trace(sys.argv[1])
