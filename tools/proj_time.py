"""Isolated timing of the dk/dv projection arms (library fp32 GEMM vs tmdnet_proj_f32) and of a plain
fill of the same output, at the C2 (8 stacked layers) and C5 (one layer) shapes.
usage: python tools/proj_time.py   (GPU box, repo root; TMDNET_PROJ_MB / _BN pick the tile)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "torchmd-net_amd"), ROOT]
import torch  # noqa: E402

from torchmdnet import kernels  # noqa: E402

dev = torch.device("cuda", 0)


def t(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for tag, M, N in (("c2", 6613, 4096), ("c5", 1361000, 512)):
    f = torch.rand(M, 64, device=dev)
    w = torch.randn(N, 64, device=dev) / 8
    b = torch.randn(N, device=dev)
    out = torch.empty(M, N, device=dev)
    reps = 20 if M > 100000 else 200
    us_lib = t(lambda: torch.addmm(b, f, w.t(), out=out), reps)
    wp = kernels.proj_split(w)
    us_x3 = t(lambda: kernels.proj(f, w, b, out=out, wp=wp), reps)
    us_fill = t(lambda: out.fill_(1.0), reps)
    gb = M * N * 4 / 1e9
    print(f"{tag} MB={os.environ.get('TMDNET_PROJ_MB', '-')} BN={os.environ.get('TMDNET_PROJ_BN', '-')} "
          f"STG={os.environ.get('TMDNET_PROJ_STG', '-')}: "
          f"lib {us_lib:.1f} us  x3 {us_x3:.1f} us  fill {us_fill:.1f} us  ({gb / us_x3 * 1e6 / 1e3:.2f} TB/s x3, "
          f"{gb / us_fill * 1e6 / 1e3:.2f} TB/s fill)", flush=True)
