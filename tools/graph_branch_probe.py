"""Do independent branches of a captured HIP graph run concurrently on this GPU?  Times a replay of
K pairs of independent small GEMMs captured on one stream vs forked over two streams (diagnosis)."""
import torch

dev = torch.device("cuda", 0)
torch.manual_seed(0)
N, H = 678, 128
a1, a2 = torch.randn(N, H, device=dev), torch.randn(3 * N, H, device=dev)
w1, w2 = torch.randn(5 * H, H, device=dev), torch.randn(3 * H, H, device=dev)
K = 16


def body(two):
    s_main = torch.cuda.current_stream()
    for _ in range(K):
        if two:
            side.wait_stream(s_main)
            torch.mm(a1, w1.t(), out=o1)
            with torch.cuda.stream(side):
                torch.mm(a2, w2.t(), out=o2)
            s_main.wait_stream(side)
        else:
            torch.mm(a1, w1.t(), out=o1)
            torch.mm(a2, w2.t(), out=o2)


o1 = torch.empty(N, 5 * H, device=dev)
o2 = torch.empty(3 * N, 3 * H, device=dev)
side = torch.cuda.Stream()
for two in (False, True):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            body(two)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body(two)
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    print(f"two_streams={two}: {e0.elapsed_time(e1) / 20 / K * 1000:.2f} us per GEMM pair")
