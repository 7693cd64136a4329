"""Capture (do NOT replay) the bench-scale training step and dump the HIP graph (diagnosis)."""
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
tr.backward(tr.loss(z, pos.clone(), batch, y, f))
cap = 15872
for d in _distance_modules(model):
    d.static_capacity = cap
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(3):
        torch.autograd.grad(tr.loss(z, pos, batch, y, f), params, allow_unused=True)
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
g.enable_debug_mode()
with torch.cuda.graph(g):
    loss = tr.loss(z, pos, batch, y, f)
    grads = torch.autograd.grad(loss, params, allow_unused=True)
torch.cuda.synchronize()
g.debug_dump(os.path.join(ROOT, "gpurun_out", "train_graph.dot"))
print("dumped", flush=True)
