"""Times tmdnet_gemm_f32 (grouped split-K MFMA) against the library GEMM on the neighbour-embedding
shapes of the C2 step (distance_proj, combine, and their input gradients)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "torchmd-net_amd"), ROOT]
import torch  # noqa: E402

from torchmdnet import kernels  # noqa: E402

dev = torch.device("cuda", 0)
E, N, R, H = 12548, 678, 64, 128
f = dict(dtype=torch.float32, device=dev)
cases = {
    "distance_proj [E x R] W^T": (torch.randn(E, R, **f), torch.randn(H, R, **f), True, torch.randn(H, **f)),
    "combine [N x 2H] W^T": (torch.randn(N, 2 * H, **f), torch.randn(H, 2 * H, **f), True, torch.randn(H, **f)),
    "combine input grad [N x H] W": (torch.randn(N, H, **f), torch.randn(H, 2 * H, **f), False, None),
    "distance_proj input grad [E x H] W": (torch.randn(E, H, **f), torch.randn(H, R, **f), False, None),
}


def timed(fn, reps=50):
    """Per-call time inside a replayed HIP graph of `reps` calls (the step runs as graph replay)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (5 * reps) * 1000


for name, (A, B, tb, bias) in cases.items():
    Bop = B.t() if tb else B
    C = torch.empty(A.shape[0], Bop.shape[1], **f)
    lib = timed(lambda: torch.addmm(bias, A, Bop, out=C) if bias is not None else torch.mm(A, Bop, out=C))
    ok = kernels.gemm_launch([(A, B, tb, bias, C, False)])
    ours = timed(lambda: kernels.gemm_launch([(A, B, tb, bias, C, False)])) if ok else float("nan")
    ref = (A.double() @ Bop.double() + (bias.double() if bias is not None else 0))
    err = ((C.double() - ref).abs().max() / ref.abs().max()).item() if ok else float("nan")
    print(f"{name:40s} library {lib:7.2f} us   tmdnet_gemm_f32 {ours:7.2f} us   rel err {err:.1e}")
