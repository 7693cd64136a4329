"""Bench-scale re-validation of training.GraphedTrainStep (ET-QM9, 32 molecules): the captured
step's loss and parameter gradients against an eager LNNPStep on an identical model copy, then
the replayed step's time.  Prints one JSON line.  usage: graphed_train_check.py [steps]"""
import copy
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "torchmd-net_amd"), ROOT]
import torch  # noqa: E402

from bench import et_args, qm9_like  # noqa: E402
from torchmdnet.models.model import create_model  # noqa: E402
from torchmdnet.training import GraphedTrainStep, LNNPStep  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = create_model(et_args(128)).to(dev)
ref_model = copy.deepcopy(model)
z, pos, batch = qm9_like(32, 1)
gy = torch.Generator().manual_seed(100)
y_lab = torch.randn(32, 1, generator=gy).to(dev)
f_lab = torch.randn(z.shape[0], 3, generator=gy).to(dev)
z, pos, batch = z.to(dev), pos.float().to(dev), batch.to(dev)

# eager reference loss / gradients on the copy
ref = LNNPStep(ref_model, lr=4e-4)
ref.opt.zero_grad(set_to_none=True)
loss_ref = ref.loss(z, pos.clone(), batch, y_lab, f_lab)
ref.backward(loss_ref)
g_ref = [p.grad.detach().clone() if p.grad is not None else torch.zeros_like(p) for p in ref.reduce.params]
torch.cuda.synchronize()
print("eager reference done", float(loss_ref), file=sys.stderr, flush=True)

gtr = GraphedTrainStep(model, z, pos, batch, y_lab, f_lab, lr=4e-4)
print("captured, capacity", gtr.edge_capacity, file=sys.stderr, flush=True)
gtr.graph.replay()
torch.cuda.synchronize()
gtr.check_capacity()
rel = lambda a, b: float((a - b).norm() / b.norm().clamp_min(1e-30))  # noqa: E731
loss_rel = abs(float(gtr.static_loss) - float(loss_ref)) / abs(float(loss_ref))
grad_rel = max(rel(a, b) for a, b in zip(gtr.reduce.views, g_ref))  # the replay writes them there
print("replay matches", loss_rel, grad_rel, file=sys.stderr, flush=True)
for _ in range(3):
    gtr.step()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(steps):
    gtr.step()
torch.cuda.synchronize()
ms = 1000 * (time.perf_counter() - t0) / steps
gtr.check_capacity()
print(json.dumps({"graphed_train_ms_per_step": round(ms, 4), "molecules_per_s": round(32 * 1000 / ms, 1),
                  "loss_rel_vs_eager": loss_rel, "max_grad_rel_vs_eager": grad_rel,
                  "edge_capacity": gtr.edge_capacity}))
