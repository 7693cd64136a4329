"""Device time of one eager ET-QM9 training step attributed to the autograd nodes that launched it
(torch.profiler; the bench workload: 32 QM9-like molecules, H=128, 8 layers, E+F MSE, AdamW).
usage (GPU box, repo root): python tools/train_node_profile.py [et_qm9|et_spice] > gpurun_out/x.txt"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "torchmd-net_amd"), ROOT]
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from bench import et_args, qm9_like  # noqa: E402
from torchmdnet.models.model import create_model  # noqa: E402
from torchmdnet.training import LNNPStep  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = create_model(et_args(128)).to(dev)
z, pos, batch = qm9_like(32, 1)
z, pos, batch = z.to(dev), pos.float().to(dev), batch.to(dev)
g = torch.Generator().manual_seed(200)
y = torch.randn(32, 1, generator=g).to(dev)
f = torch.randn(z.shape[0], 3, generator=g).to(dev)
step = LNNPStep(model, lr=1e-4)
for _ in range(3):
    step.step(z, pos, batch, y, f)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    step.step(z, pos, batch, y, f)
    torch.cuda.synchronize()
ev = prof.key_averages()
rows = []
for e in ev:
    t = getattr(e, "device_time_total", None) or getattr(e, "cuda_time_total", 0)
    if e.key.startswith("autograd::engine::evaluate_function") or e.key in ("aten::mse_loss",):
        rows.append((t, e.count, e.key))
tot = sum(getattr(e, "self_device_time_total", 0) or getattr(e, "self_cuda_time_total", 0) for e in ev)
print(f"total device time {tot / 1000:.3f} ms")
for t, c, k in sorted(rows, reverse=True)[:40]:
    print(f"{t / 1000:9.3f} ms {c:4d}  {k[:110]}")
print()
print(ev.table(sort_by="self_cuda_time_total" if hasattr(ev[0], "self_cuda_time_total") else "self_device_time_total",
               row_limit=40, max_name_column_width=90))
print()
# the GEMM / reduction ops with their input shapes (which call site is the expensive one)
gs = prof.key_averages(group_by_input_shape=True)
rows = []
for e in gs:
    if e.key in ("aten::mm", "aten::addmm", "aten::bmm", "aten::baddbmm", "aten::addmm_", "aten::sum", "aten::mul",
                 "aten::add", "aten::add_", "aten::index_select", "aten::index_add_", "aten::embedding_backward",
                 "aten::embedding_dense_backward", "aten::fill_", "aten::copy_", "aten::cat", "aten::zeros"):
        t = getattr(e, "device_time_total", None) or getattr(e, "cuda_time_total", 0)
        rows.append((t, e.count, e.key, str(e.input_shapes)[:150]))
for t, c, k, sh in sorted(rows, reverse=True)[:45]:
    print(f"{t / 1000:9.3f} ms {c:4d}  {k:24s} {sh}")
