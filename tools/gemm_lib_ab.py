"""Time the ET-QM9 node-GEMM shapes under hipBLASLt and rocBLAS (torch's preferred BLAS switch)."""
import torch

dev = torch.device("cuda", 0)
shapes = [  # (op, M, K, N): out[M,N] = A[M,K] @ B[K,N] (+ bias)
    ("addmm", 678, 128, 640), ("mm", 2034, 128, 384), ("addmm", 678, 128, 384),
    ("mm", 678, 640, 128), ("mm", 678, 384, 128), ("addmm_", 2034, 384, 128),
    ("addmm", 12548, 64, 4096), ("mm", 12548, 4096, 64),
]


def bench(fn, reps=50):
    """GPU time per call: the calls are captured in a HIP graph (no host launch overhead)."""
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
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(4):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / (4 * reps)


for lib in ("cublaslt", "cublas"):
    try:
        torch.backends.cuda.preferred_blas_library(lib)
    except Exception as e:  # noqa: BLE001
        print(lib, "unavailable", e)
        continue
    print("library", torch.backends.cuda.preferred_blas_library())
    for op, M, K, N in shapes:
        A = torch.randn(M, K, device=dev)
        W = torch.randn(N, K, device=dev)
        bias = torch.randn(N, device=dev)
        C = torch.randn(M, N, device=dev)
        if op == "addmm":
            fn = lambda: torch.addmm(bias, A, W.t())  # noqa: E731
        elif op == "mm":
            fn = lambda: A @ W.t()  # noqa: E731
        else:
            fn = lambda: C.addmm_(A, W.t())  # noqa: E731
        print(f"  {op:7s} M={M:6d} K={K:5d} N={N:5d}  {bench(fn):7.2f} us")
