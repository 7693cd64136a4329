"""The explicit second-order neighbour formulas (kernels.nl_backward2_composite, the restatement
tmdnet_nl_backward2 implements) equal autograd through the first-order composite, CPU fp64, on a
symmetric list with self loops, zero-distance pairs and static-capacity padding slots."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "torchmd-net_amd"))
from torchmdnet import kernels  # noqa: E402


def _graph(n=12, cap_pad=7, seed=0):
    g = torch.Generator().manual_seed(seed)
    pos = torch.rand(n, 3, generator=g, dtype=torch.float64) * 3
    pos[5] = pos[4]  # a coincident pair: r == 0 on a non-self edge
    pairs = [(i, j) for i in range(n) for j in range(n) if i != j and torch.rand(1, generator=g) < 0.4]
    pairs += [(i, i) for i in range(n)]
    if (4, 5) not in pairs:
        pairs += [(4, 5), (5, 4)]
    pairs = sorted(set(pairs) | {(j, i) for i, j in pairs})
    src = torch.tensor([p[0] for p in pairs] + [-1] * cap_pad, dtype=torch.int32)
    dst = torch.tensor([p[1] for p in pairs] + [-1] * cap_pad, dtype=torch.int32)
    s, d = src.long().clamp(min=0), dst.long().clamp(min=0)
    dl = (pos[s] - pos[d]) * (src >= 0).unsqueeze(1)
    r = dl.norm(dim=1)
    return pos, src, dst, dl, r


def test_second_order_formula_matches_autograd():
    pos, src, dst, dl, r = _graph()
    E = src.shape[0]
    g = torch.Generator().manual_seed(1)
    gd = torch.randn(E, 3, generator=g, dtype=torch.float64)
    gr = torch.randn(E, generator=g, dtype=torch.float64)
    gg = torch.randn(pos.shape, generator=g, dtype=torch.float64)
    p = pos.clone().requires_grad_(True)
    gd_ = gd.clone().requires_grad_(True)
    gr_ = gr.clone().requires_grad_(True)
    out = kernels.nl_backward_composite(p, gd_, gr_, dl, r, src, dst)
    ref = torch.autograd.grad(out, (p, gd_, gr_), gg)
    d_pos, d_gd, d_gr = kernels.nl_backward2_composite(pos, gg, gr, dl, r, src, dst)
    for a, b in zip((d_pos, d_gd, d_gr), ref):
        assert torch.allclose(a, b, rtol=1e-12, atol=1e-12)
    # padding slots and r == 0 edges carry nothing
    dead = (src < 0) | (r == 0)
    assert torch.all(d_gd[dead] == 0) and torch.all(d_gr[dead] == 0)


def test_second_order_without_distance_gradient():
    pos, src, dst, dl, r = _graph(seed=3)
    E = src.shape[0]
    gd = torch.randn(E, 3, dtype=torch.float64)
    gg = torch.randn(pos.shape, dtype=torch.float64)
    p = pos.clone().requires_grad_(True)
    gd_ = gd.clone().requires_grad_(True)
    out = kernels.nl_backward_composite(p, gd_, None, dl, r, src, dst)
    ref = torch.autograd.grad(out, (p, gd_), gg, allow_unused=True)
    d_pos, d_gd, _ = kernels.nl_backward2_composite(pos, gg, None, dl, r, src, dst)
    assert ref[0] is None or torch.allclose(ref[0], torch.zeros_like(ref[0]))
    assert torch.all(d_pos == 0)
    assert torch.allclose(d_gd, ref[1], rtol=1e-12, atol=1e-12)
