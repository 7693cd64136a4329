"""Time the fused head kernel (forward + Jacobian) at the C2 atom count and at C5 scale."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "torchmd-net_amd"), ROOT]
import torch  # noqa: E402
from torchmdnet import kernels  # noqa: E402
from torchmdnet.models.output_modules import EquivariantScalar  # noqa: E402

dev = torch.device("cuda", 0)
for N in (580, 4096, 50000):
    H = 128
    head = EquivariantScalar(H).to(dev)
    x = torch.randn(N, H, device=dev, requires_grad=True)
    v = torch.randn(N, 3, H, device=dev, requires_grad=True)
    for _ in range(5):
        y = kernels.eq_scalar_head(x, v, head.output_network)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 50
    a.record()
    for _ in range(reps):
        y = kernels.eq_scalar_head(x, v, head.output_network)
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) * 1000 / reps
    print(f"N={N} head fwd+J {us:.1f} us  ({us / N * 1000:.1f} ns/atom)", flush=True)
