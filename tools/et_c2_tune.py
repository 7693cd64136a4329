"""ET message fwd / bwd kernel time at C2 size (32 QM9-like molecules, H=128, 8 heads), measured
from a HIP graph of back-to-back launches (no host overhead); env variants (TMDNET_ET_S) A/B."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "torchmd-net_amd"), ROOT, os.path.join(ROOT, "tools")]
import torch  # noqa: E402
from torchmdnet import kernels  # noqa: E402
from kbench import graph_c2, et_inputs, _Ctx  # noqa: E402


def graphed(fn, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
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
    for _ in range(5):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / (5 * reps)


dev = torch.device("cuda", 0)
g = graph_c2(dev)
x = et_inputs(g, 128, dev)
args = [x[k] for k in ("q", "k", "v", "vec", "pk", "pv", "C", "u")]
N = g.n_nodes
gx, gv = torch.randn(N, 128, device=dev), torch.randn(N, 3, 128, device=dev)
for var in (sys.argv[1:] or [""]):
    if var:
        k, v = var.split("=")
        os.environ[k] = v
    tf = graphed(lambda: kernels._ETMessage.forward(_Ctx(), *args, g, 8))
    tb = graphed(lambda: kernels._ETMessageBwd.forward(_Ctx(), gx, gv, *args, g, 8))
    print(f"C2 N={N} E={g.n_edges} {var or 'default'}: fwd {tf:6.1f} us  bwd {tb:6.1f} us", flush=True)
