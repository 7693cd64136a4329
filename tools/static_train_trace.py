"""Eager bench-scale training step with the static-capacity neighbour list (the ops a captured step
replays), bracketed by marker kernels for rocprofv3 (diagnosis)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "torchmd-net_amd"), ROOT]
import torch  # noqa: E402
from bench import et_args, qm9_like  # noqa: E402
from torchmdnet.models.model import create_model  # noqa: E402
from torchmdnet.training import LNNPStep  # noqa: E402
from torchmdnet.graphs import _distance_modules  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = create_model(et_args(128)).to(dev)
z, pos, batch = qm9_like(32, 1)
z, pos, batch = z.to(dev), pos.float().to(dev), batch.to(dev)
y = torch.randn(32, 1, device=dev)
f = torch.randn(z.shape[0], 3, device=dev)
tr = LNNPStep(model, lr=4e-4)
params = tr.reduce.params
for d in _distance_modules(model):
    d.static_capacity = 15872
for _ in range(2):
    torch.autograd.grad(tr.loss(z, pos, batch, y, f), params, allow_unused=True)
torch.cuda.synchronize()
print("eager static ok", flush=True)
torch.cuda._sleep(100)
torch.autograd.grad(tr.loss(z, pos, batch, y, f), params, allow_unused=True)
torch.cuda._sleep(100)
torch.cuda.synchronize()
print("traced", flush=True)

if os.environ.get("STT_PROFILE"):
    from torch.profiler import profile, ProfilerActivity
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True,
                 with_stack=True) as prof:
        torch.autograd.grad(tr.loss(z, pos, batch, y, f), params, allow_unused=True)
        torch.cuda.synchronize()
    prof.export_chrome_trace(os.environ["STT_PROFILE"])
