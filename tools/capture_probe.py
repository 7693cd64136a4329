"""Which part of a training step breaks HIP-graph capture?  One mode per process:
energy | force_perlayer | force_fused  [relaxed]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "torchmd-net_amd"), ROOT, os.path.join(ROOT, "tests")]
import torch  # noqa: E402
from conftest import yaml_args  # noqa: E402
from oracle import model_oracle as O  # noqa: E402
from torchmdnet.models.model import create_model  # noqa: E402
from torchmdnet.graphs import _distance_modules  # noqa: E402

mode = sys.argv[1]
err_mode = sys.argv[2] if len(sys.argv) > 2 else "global"
DEV = torch.device("cuda", 0)
torch.manual_seed(0)
m = create_model(yaml_args("equivariant-transformer", embedding_dimension=32, num_layers=2, num_rbf=16,
                           num_heads=4, derivative=True, output_model="Scalar")).to(DEV)
m.representation_model.fused_stack = mode != "force_perlayer"
z, pos, batch = O.qm9_like(4)
z, pos, batch = z.to(DEV), pos.float().to(DEV), batch.to(DEV)
y_lab = torch.randn(4, 1, device=DEV)
f_lab = torch.randn(pos.shape, device=DEV)
params = [p for p in m.parameters() if p.requires_grad]


def loss_fn():
    y, f = m(z, pos, batch)
    loss = ((y - y_lab) ** 2).mean()
    if mode != "energy":
        loss = loss + ((f - f_lab) ** 2).mean()
    return loss


pos0 = pos
pos = pos0.clone()
torch.autograd.grad(loss_fn(), params, allow_unused=True)
pos = pos0
for d in _distance_modules(m):
    d.static_capacity = 4096
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(3):
        torch.autograd.grad(loss_fn(), params, allow_unused=True)
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
print("warm-up ok", flush=True)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, capture_error_mode=err_mode):
    loss = loss_fn()
    grads = torch.autograd.grad(loss, params, allow_unused=True)
print("capture ok", flush=True)
g.replay()
torch.cuda.synchronize()
print("replay ok", float(loss), flush=True)
