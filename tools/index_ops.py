"""List aten index-family calls (with shapes) of one eager ET training step (diagnosis tool)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "torchmd-net_amd"), ROOT, os.path.join(ROOT, "tests")]
import torch  # noqa: E402
from conftest import yaml_args  # noqa: E402
from oracle import model_oracle as O  # noqa: E402
from torchmdnet.models.model import create_model  # noqa: E402
from torchmdnet.training import LNNPStep  # noqa: E402

DEV = torch.device("cuda", 0)
torch.manual_seed(0)
m = create_model(yaml_args("equivariant-transformer", embedding_dimension=32, num_layers=2, num_rbf=16,
                           num_heads=4, derivative=True, output_model="Scalar")).to(DEV)
z, pos, batch = O.qm9_like(4)
z, pos, batch = z.to(DEV), pos.float().to(DEV), batch.to(DEV)
y = torch.randn(4, 1, device=DEV)
f = torch.randn(pos.shape, device=DEV)
tr = LNNPStep(m, lr=1e-4)
tr.step(z, pos, batch, y, f)
torch.cuda.synchronize()
print("E =", m.representation_model.distance.last_num_pairs, "N =", z.shape[0])
from torch.profiler import profile, ProfilerActivity  # noqa: E402
with profile(activities=[ProfilerActivity.CPU], record_shapes=True) as prof:
    tr.step(z, pos, batch, y, f)
    torch.cuda.synchronize()
for ev in prof.events():
    if ev.name in ("aten::index", "aten::index_put_", "aten::_index_put_impl_", "aten::index_put",
                   "aten::as_strided_scatter", "aten::masked_select", "aten::take"):
        print(ev.name, ev.input_shapes)
