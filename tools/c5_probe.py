"""Run only the ET message forward on the C5-scale water box (for PMC counter passes)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "torchmd-net_amd"), ROOT, os.path.join(ROOT, "tools")]
import torch  # noqa: E402
from torchmdnet import kernels  # noqa: E402
from kbench import graph_c5, et_inputs, _Ctx  # noqa: E402

order = sys.argv[1] if len(sys.argv) > 1 else "morton"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
dev = torch.device("cuda", 0)
g = graph_c5(50001, dev, order)
x = et_inputs(g, 128, dev)
args = [x[k] for k in ("q", "k", "v", "vec", "pk", "pv", "C", "u")]
for _ in range(reps):
    kernels._ETMessage.forward(_Ctx(), *args, g, 8)
torch.cuda.synchronize()
print("E", g.n_edges, "N", g.n_nodes)
