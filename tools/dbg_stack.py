"""Debug: fused stack first backward (opaque vs differentiable recompute) vs per-layer path."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "torchmd-net_amd"), ROOT, os.path.join(ROOT, "tests")]
import torch  # noqa: E402
from conftest import yaml_args  # noqa: E402
from oracle import model_oracle as O  # noqa: E402
from torchmdnet.models.model import create_model  # noqa: E402
from torchmdnet import et_stack as ES  # noqa: E402

DEV = torch.device("cuda", 0)
torch.manual_seed(1234)
for H, heads, prec in ((32, 4, 64), (64, 4, 64), (128, 8, 32)):
    m = create_model(yaml_args("equivariant-transformer", embedding_dimension=H, num_layers=2, num_rbf=16,
                               num_heads=heads, derivative=True, output_model="Scalar", precision=prec)).to(DEV)
    z, pos, batch = O.qm9_like(3)
    dt = torch.float64 if prec == 64 else torch.float32
    z, pos, batch = z.to(DEV), pos.to(dt).to(DEV), batch.to(DEV)
    res = {}
    for mode in ("perlayer", "fused"):
        m.representation_model.fused_stack = mode == "fused"
        y, f = m(z, pos.clone(), batch)
        res[mode] = (y.detach(), f.detach())
    for mode in ("fused",):
        print(H, heads, prec, "y", (res[mode][0] - res["perlayer"][0]).abs().max().item(),
              "f", (res[mode][1] - res["perlayer"][1]).abs().max().item(), res["perlayer"][1].abs().max().item())
