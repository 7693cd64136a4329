"""Which Python call launches the fill kernels of an ET-QM9 energy + force evaluation (eager, after a
warm-up): wraps the torch factory / fill functions and prints the caller of every CUDA one."""
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "torchmd-net_amd"), ROOT]
import torch  # noqa: E402
import yaml  # noqa: E402
from torchmdnet.models.model import create_model  # noqa: E402

with open(os.path.join(ROOT, "tests", "golden", "configs", "et_qm9.yaml")) as f:
    args = yaml.safe_load(f)
args.update(prior_model=None, embedding_dimension=128, derivative=True)
torch.manual_seed(0)
model = create_model(args).cuda()
g = torch.Generator().manual_seed(1)
sizes = torch.randint(12, 29, (32,), generator=g)
batch = torch.repeat_interleave(torch.arange(32), sizes)
z = torch.tensor([1, 6, 7, 8])[torch.randint(0, 4, (int(sizes.sum()),), generator=g)]
pos = torch.rand(int(sizes.sum()), 3, generator=g) * 4.0
z, pos, batch = z.cuda(), pos.float().cuda(), batch.cuda()
for _ in range(2):
    model(z, pos.clone(), batch)
torch.cuda.synchronize()
active = [True]


def wrap(mod, name):
    orig = getattr(mod, name)

    def f(*a, **k):
        out = orig(*a, **k)
        dev = k.get("device")
        is_cuda = (isinstance(out, torch.Tensor) and out.is_cuda) or (dev is not None and "cuda" in str(dev))
        if active[0] and is_cuda:
            print("==", name, tuple(out.shape) if isinstance(out, torch.Tensor) else "")
            print("".join(traceback.format_stack(limit=5)[:-1]))
        return out
    setattr(mod, name, f)


for n in ("zeros", "zeros_like", "ones", "ones_like", "full", "full_like"):
    wrap(torch, n)
for n in ("fill_", "zero_"):
    wrap(torch.Tensor, n)
model(z, pos.clone(), batch)
torch.cuda.synchronize()
print("done")
