"""Debug: composite_stack with the HIP message Functions vs the PyTorch restatement."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "torchmd-net_amd"), ROOT, os.path.join(ROOT, "tests")]
import torch  # noqa: E402
from oracle import model_oracle as O  # noqa: E402
from torchmdnet import et_stack as ES, kernels  # noqa: E402
from torchmdnet.models.torchmd_et import EquivariantMultiHeadAttention  # noqa: E402

DEV = torch.device("cuda", 0)
torch.manual_seed(0)
DT = torch.float64
z, pos, batch = O.qm9_like(3)
pos = pos.to(DEV)
g = kernels.build_graph(pos, batch.to(DEV), 0.0, 5.0, 64 * pos.shape[0], loop=True)
N, E, H, R, heads = pos.shape[0], g.n_edges, 32, 16, 4
layers = torch.nn.ModuleList([EquivariantMultiHeadAttention(H, R, "both", heads, torch.nn.SiLU, "silu", 0.0, 5.0, DT)
                              for _ in range(2)]).to(DEV)
r = g.distances.detach()
f = torch.exp(-(r[:, None] - torch.linspace(0, 5, R, device=DEV, dtype=DT)) ** 2).requires_grad_(True)
C = (0.5 * (torch.cos(r * 3.14159 / 5) + 1)).requires_grad_(True)
u = (g.deltas.detach() / torch.where(r > 0, r, torch.ones_like(r))[:, None]).requires_grad_(True)
x = torch.randn(N, H, device=DEV, dtype=DT).requires_grad_(True)
params = [p for l in layers for p in ES.layer_params(l)]
meta = ES._Meta(g, heads, H, True, True, 2, None, None)
msg = lambda q, k, v, vec, pk, pv, C_, u_: kernels.et_message(q, k, v, vec, pk, pv, C_, u_, g, heads)  # noqa
a = ES.composite_stack(meta, x, f, C, u, params, message=msg)
b = ES.composite_stack(meta, x, f, C, u, params)
print("fwd", [(ai - bi).abs().max().item() for ai, bi in zip(a, b)])
gx, gv = torch.randn_like(a[0]), torch.randn_like(a[1])
ga = torch.autograd.grad(a, [x, f, C, u], (gx, gv))
gb = torch.autograd.grad(b, [x, f, C, u], (gx, gv))
T = g.transpose.long()
for n, p_, q_ in zip("x f C u".split(), ga, gb):
    d = (p_ - q_).abs().max().item()
    if n in ("f", "C"):
        ds = ((p_ + p_[T]) - (q_ + q_[T])).abs().max().item()
    elif n == "u":
        ds = ((p_ - p_[T]) - (q_ - q_[T])).abs().max().item()
    else:
        ds = d
    print(n, "direct", d, "pair-symmetrised", ds, "scale", q_.abs().max().item())
for cg in (False, True):
    xo, vo = ES.et_stack(layers, x, g, f, C, u)
    gs = torch.autograd.grad((xo, vo), [x, f, C, u], (gx, gv), create_graph=cg)
    for n, p_, q_ in zip("x f C u".split(), gs, gb):
        if n in ("f", "C"):
            ds = ((p_ + p_[T]) - (q_ + q_[T])).abs().max().item()
        elif n == "u":
            ds = ((p_ - p_[T]) - (q_ - q_[T])).abs().max().item()
        else:
            ds = (p_ - q_).abs().max().item()
        print("et_stack create_graph", cg, n, ds)
