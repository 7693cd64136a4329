"""Edge-feature gradient of the batched dk/dv projection, g_f = g_pkv_all [E, L*D] @ W [L*D, R]:
one GEMM (K = L*D = 4096, hipBLASLt picks ~196 workgroups with a 32-step K loop) vs split by layer
(bmm over L strided views, then a sum over L) -- HIP-event timed (diagnosis)."""
import torch

dev = torch.device("cuda", 0)
E, L, D, R = 12548, 8, 512, 64
g = torch.randn(E, L * D, device=dev)
w = torch.randn(L * D, R, device=dev)


def one():
    return torch.mm(g, w)


def split():
    return torch.bmm(g.view(E, L, D).transpose(0, 1), w.view(L, D, R)).sum(0)


def split_out(buf=torch.empty(L, E, R, device=dev)):
    torch.bmm(g.view(E, L, D).transpose(0, 1), w.view(L, D, R), out=buf)
    return buf.sum(0)


for name, fn in (("one", one), ("split", split), ("split_out", split_out)):
    for _ in range(5):
        r = fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print(name, f"{e0.elapsed_time(e1) / 50 * 1000:.1f} us", float((r - one()).abs().max()))
# forward: f [E, R] @ W^T -> [E, L*D] (+ bias), one GEMM vs per-layer bmm into a strided output
f = torch.randn(E, R, device=dev)
wt = torch.randn(L * D, R, device=dev)
b = torch.randn(L * D, device=dev)
out = torch.empty(E, L * D, device=dev)


def fwd_one():
    torch.addmm(b, f, wt.t(), out=out)


def fwd_bmm():
    torch.baddbmm(b.view(L, 1, D), f.unsqueeze(0).expand(L, E, R), wt.view(L, D, R).transpose(1, 2),
                  out=out.view(E, L, D).transpose(0, 1))


for name, fn in (("fwd_one", fwd_one), ("fwd_bmm", fwd_bmm)):
    try:
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            fn()
        e1.record()
        torch.cuda.synchronize()
        print(name, f"{e0.elapsed_time(e1) / 50 * 1000:.1f} us")
    except RuntimeError as ex:
        print(name, "failed:", str(ex)[:200])
