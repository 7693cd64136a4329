"""Diagnostic: TensorNet on a periodic water box, GPU vs the fp64 oracle with static_shapes on / off
(tests/test_gpu_periodic_oracle.py's TensorNet case): where the force error sits."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "torchmd-net_amd"), ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from conftest import yaml_args  # noqa: E402
from oracle import model_oracle as O  # noqa: E402
from torchmdnet import kernels  # noqa: E402
from torchmdnet.models.model import create_model  # noqa: E402


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max())


n = int(sys.argv[1]) if len(sys.argv) > 1 else 1500
periodic = len(sys.argv) <= 2 or sys.argv[2] != "open"
g = torch.Generator().manual_seed(3)
L = (n / 0.1003) ** (1.0 / 3.0)
pos = torch.rand(n, 3, generator=g, dtype=torch.float64) * L
z = torch.tensor([8, 1, 1], dtype=torch.long).repeat(n // 3 + 1)[:n]
batch = torch.zeros(n, dtype=torch.long)
kernels.REORDER_MIN_ATOMS = 10 ** 9
args = yaml_args("tensornet", embedding_dimension=128, num_layers=2, num_rbf=32, cutoff_upper=4.5,
                 max_num_neighbors=64, derivative=True, static_shapes=False)
torch.manual_seed(0)
m = create_model(args)
cfg = dict(args)
if periodic:
    cfg["box"] = np.eye(3) * L
refs = {s: O.energy_forces(m.state_dict(), cfg, z, pos, batch, static_shapes=s) for s in (False, True)}
m = m.cuda()
d = m.representation_model.distance
if periodic:
    d.box = torch.eye(3, dtype=torch.float32) * L
    d.use_periodic = True
    d.strategy = "cell"
for static in (False, True):
    m.representation_model.static_shapes = static
    y, f = m(z.cuda(), pos.float().cuda(), batch.cuda())
    for rs, (y_ref, f_ref) in refs.items():
        err = (f.detach().double().cpu() - f_ref.detach()).abs().max(dim=1).values
        bad = torch.nonzero(err > 1e-3 * f_ref.abs().max()).flatten()
        print(f"gpu static={static} vs oracle static={rs}: energy {rel(y, y_ref):.3e} forces {rel(f, f_ref):.3e} "
              f"bad atoms {bad.numel()} first {bad[:12].tolist()}", flush=True)
gr = kernels.build_graph(pos.float().cuda(), batch.cuda(), 0.0, 4.5, 64 * n, loop=True, strategy="cell" if periodic else "brute",
                         box=d.box if periodic else None)
deg = torch.diff(gr.row_ptr.long()).cpu()
print("pairs", gr.n_edges, "max degree", int(deg.max()), "num_pairs", gr.num_pairs, flush=True)
