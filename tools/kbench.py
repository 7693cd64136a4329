"""Kernel micro-benchmark (GPU): ET message fwd / bwd and TN kernels at C2 (32 QM9-like molecules)
and C5 (50k-atom water box) scale, HIP-event timed, with a correctness check against the composite
PyTorch restatement.  Usage: python tools/kbench.py [--c5-atoms N] [--reps R]"""
import argparse
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "torchmd-net_amd"), ROOT]
import torch  # noqa: E402
from torchmdnet import kernels  # noqa: E402
if os.environ.get("KBENCH_LIB"):  # A/B against another build (tools/build_ab.sh)
    kernels.nat._LIB_PATH = os.path.abspath(os.environ["KBENCH_LIB"])
from bench import qm9_like, et_algorithmic_bytes  # noqa: E402


def graph_c2(dev):
    z, pos, batch = qm9_like(32, 1)
    return kernels.build_graph(pos.float().to(dev), batch.to(dev), 0.0, 5.0, 64 * len(z), loop=True)


def morton3(c):
    def spread(x):
        x = x & 0x3FF
        x = (x | (x << 16)) & 0x030000FF
        x = (x | (x << 8)) & 0x0300F00F
        x = (x | (x << 4)) & 0x030C30C3
        x = (x | (x << 2)) & 0x09249249
        return x
    return spread(c[:, 0]) | (spread(c[:, 1]) << 1) | (spread(c[:, 2]) << 2)


def graph_c5(n, dev, order="cell"):
    g = torch.Generator().manual_seed(7)
    L = (n / 0.1003) ** (1 / 3)
    pos = (torch.rand(n, 3, generator=g, dtype=torch.float64) * L).float()
    # renumber atoms in cell order (spatially coherent numbering, as MD engines / PDB files give)
    nc = max(3, int(L / 5.0))
    cell = torch.clamp((pos / (L / nc)).long(), 0, nc - 1)
    if order == "morton":
        key = morton3(cell)
    elif order == "random":
        key = torch.randperm(n, generator=g)
    else:
        key = (cell[:, 2] * nc + cell[:, 1]) * nc + cell[:, 0]
    pos = pos[torch.argsort(key)].contiguous().to(dev)
    return kernels.build_graph(pos, torch.zeros(n, dtype=torch.long, device=dev), 0.0, 5.0, 128 * n,
                               loop=True, strategy="cell", box=torch.eye(3) * L)


def timeit(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3  # us


def et_inputs(g, H, dev):
    N, E = g.n_nodes, g.n_edges
    gen = torch.Generator(device=dev).manual_seed(3)
    rn = lambda *s: torch.randn(*s, device=dev, generator=gen)
    T = g.transpose.long()
    sym = lambda x: ((x + x[T]) * 0.5).contiguous()
    r = g.distances.detach()
    C = 0.5 * (torch.cos(r * math.pi / 5.0) + 1.0)
    u = (g.deltas.detach() / torch.where(r > 0, r, torch.ones_like(r)).unsqueeze(1)).contiguous()
    return dict(q=rn(N, H), k=rn(N, H), v=rn(N, 3 * H), vec=rn(N, 3, H), pk=sym(rn(E, H)), pv=sym(rn(E, 3 * H)),
                C=C, u=u)


def run_et(name, g, H, reps, dev, check):
    x = et_inputs(g, H, dev)
    args = [x[k] for k in ("q", "k", "v", "vec", "pk", "pv", "C", "u")]
    N, E = g.n_nodes, g.n_edges
    fwd = lambda: kernels._ETMessage.forward(_Ctx(), *args, g, 8)
    gx, gv = torch.randn(N, H, device=dev), torch.randn(N, 3, H, device=dev)
    bwd = lambda: kernels._ETMessageBwd.forward(_Ctx(), gx, gv, *args, g, 8)
    tf = timeit(fwd, reps)
    tb = timeit(bwd, reps)
    B = et_algorithmic_bytes(E, N, H)
    print(f"{name}: N={N} E={E}  fwd {tf:8.1f} us {B / tf / 1e3:7.1f} GB/s ({B / tf / 1e3 / 80:5.1f}%)  "
          f"bwd(dst+src) {tb:8.1f} us")
    if check:
        xo, vo = fwd()
        xr, vr = kernels.et_message_composite(*args, g.src.long(), g.dst.long(), N, 8)
        e1 = ((xo - xr).abs().max() / xr.abs().max()).item()
        e2 = ((vo - vr).abs().max() / vr.abs().max()).item()
        outs = bwd()
        ins = [a.detach().requires_grad_(True) for a in args]
        with torch.enable_grad():
            xr, vr = kernels.et_message_composite(*ins, g.src.long(), g.dst.long(), N, 8)
            ref = torch.autograd.grad((xr, vr), ins, (gx, gv))
        T = g.transpose.long()
        errs = []
        for nm, a, b in zip("q k v vec pk pv C u".split(), outs, ref):
            if nm in ("pk", "pv", "C"):
                a, b = a + a[T], b + b[T]
            if nm == "u":
                a, b = a - a[T], b - b[T]
            errs.append(((a - b).abs().max() / b.abs().max().clamp(min=1e-30)).item())
        print(f"   check fwd {e1:.1e} {e2:.1e}  bwd max rel {max(errs):.1e}")
        assert max(e1, e2, max(errs)) < 1e-4


class _Ctx:
    def save_for_backward(self, *a):
        pass


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--c5-atoms", type=int, default=50001)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--no-c5", action="store_true")
    ap.add_argument("--variants", default="", help="comma list of ENV=value kernel switches to A/B")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g2 = graph_c2(dev)
    variants = [v for v in a.variants.split(",") if v]
    for var in variants or [""]:
        if var:
            k, val = var.split("=")
            os.environ[k] = val
        run_et(f"C2 ET {var}", g2, 128, 200, dev, True)
    if not a.no_c5:
        g5 = graph_c5(a.c5_atoms, dev, "morton")
        for var in variants or [""]:
            if var:
                k, val = var.split("=")
                os.environ[k] = val
            run_et(f"C5 ET morton {var}", g5, 128, a.reps, dev, True)

if __name__ == "__main__" and not os.environ.get("KBENCH_DECOMPOSE"):
    main()


def decompose(g, H, reps, dev, heads=8):
    """C5 fwd time split: full / no per-edge stream (pk=pv=None) / gathers from own row only."""
    x = et_inputs(g, H, dev)
    N = g.n_nodes
    xo = torch.empty(N, H, device=dev)
    vo = torch.empty(N, 3, H, device=dev)
    full = lambda gr, pk, pv: kernels.et_message_fwd_launch(x["q"], x["k"], x["v"], x["vec"], pk, pv, x["C"],  # noqa
                                                           x["u"], gr, heads, xo, vo)
    t_full = timeit(lambda: full(g, x["pk"], x["pv"]), reps)
    t_nostream = timeit(lambda: full(g, None, None), reps)
    import copy
    g_self = copy.copy(g)
    g_self.src = g.dst.clone()  # every gather hits the destination's own row (perfect locality)
    t_self = timeit(lambda: full(g_self, x["pk"], x["pv"]), reps)
    t_self_ns = timeit(lambda: full(g_self, None, None), reps)
    E = g.n_edges
    t_sum = timeit(lambda: (x["pk"].sum(), x["pv"].sum()), reps)
    buf = torch.empty(E * 4 * H, device=dev)
    t_copy = timeit(lambda: (buf[:E * H].copy_(x["pk"].view(-1)), buf[E * H:].copy_(x["pv"].view(-1))), reps)
    print(f"   plain torch over the same stream: sum {t_sum:.0f} us ({E * 16 * H / t_sum / 1e3:.0f} GB/s read), "
          f"copy {t_copy:.0f} us ({2 * E * 16 * H / t_copy / 1e3:.0f} GB/s r+w)")
    print(f"decompose heads={heads} N={N} E={E}: full {t_full:.0f} us | no dk/dv stream {t_nostream:.0f} us | "
          f"self-gathers {t_self:.0f} us | self-gathers, no stream {t_self_ns:.0f} us | "
          f"stream bytes {E * 16 * H / 1e9:.2f} GB")


if __name__ == "__main__" and os.environ.get("KBENCH_DECOMPOSE"):
    _dev = torch.device("cuda", 0)
    _g = graph_c5(50001, _dev, "morton")
    for _h in (8, 2, 1):
        decompose(_g, 128, 20, _dev, _h)
    # interleaved vs planar v / dv rows, same graph, alternating
    x = et_inputs(_g, 128, _dev)
    N = _g.n_nodes
    xo, vo = torch.empty(N, 128, device=_dev), torch.empty(N, 3, 128, device=_dev)
    for rep_ in range(3):
        for fl in (0, 4):
            t = timeit(lambda: kernels.et_message_fwd_launch(x["q"], x["k"], x["v"], x["vec"], x["pk"], x["pv"],
                                                             x["C"], x["u"], _g, 8, xo, vo, fl), 20)
            print(f"fwd flags={fl}: {t:.0f} us")
