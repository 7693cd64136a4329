"""Stage-by-stage TensorNet comparison on the GPU: each HIP launch vs its PyTorch composite inside a
real model forward (diagnosis)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "torchmd-net_amd"), ROOT, os.path.join(ROOT, "tests")]
import torch  # noqa: E402

from torchmdnet import kernels, tn_node  # noqa: E402
import test_tn_node_cpu as E  # noqa: E402
from conftest import yaml_args  # noqa: E402
from oracle import model_oracle as O  # noqa: E402
from torchmdnet.models.model import create_model  # noqa: E402

torch.manual_seed(0)
m = create_model(yaml_args("tensornet", output_model="Scalar", derivative=False)).to("cuda").double()
m.representation_model.static_shapes = False
z, pos, batch = O.qm9_like(3)
z, pos, batch = z.cuda(), pos.double().cuda(), batch.cuda()

pairs = [("node_fwd_launch", tn_node, E._fake_node_fwd), ("tn_embed_fwd_launch", kernels, E._fake_embed_fwd),
         ("tn_message_fwd_launch", kernels, E._fake_msg_fwd)]
for name, mod, fake in pairs:
    real = getattr(mod, name)

    def wrapped(*args, _real=real, _fake=fake, _name=name):
        out = args[-1]
        _real(*args)
        torch.cuda.synchronize()
        got = out.clone()
        _fake(*args)
        err = (got - out).abs().max().item() / max(out.abs().max().item(), 1e-30)
        print(f"{_name} {args[0] if _name == 'node_fwd_launch' else ''}: rel err {err:.3e}")
    setattr(mod, name, wrapped)
with torch.no_grad():
    y = m(z, pos, batch)
