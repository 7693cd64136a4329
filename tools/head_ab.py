"""A/B of the equivariant head's two kernels (the bf16-MFMA 16-atom-tile form vs the per-atom VALU form),
forward + Jacobian, µs per call (graph-replayed) at several atom counts: picks kernels.HEAD_X3_MIN_ATOMS.
usage (GPU box, repo root): python3 tools/head_ab.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "torchmd-net_amd")]
import torch  # noqa: E402


def main():
    from torchmdnet import kernels
    from torchmdnet.models.output_modules import EquivariantScalar
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    head = EquivariantScalar(128).to(dev)
    out = {}
    for n in (678, 1024, 2048, 4096, 8192, 16384, 50000):
        x = torch.randn(n, 128, device=dev, requires_grad=True)
        v = torch.randn(n, 3, 128, device=dev, requires_grad=True)
        row = {}
        for x3 in (True, False):
            kernels.HEAD_X3, kernels.HEAD_X3_MIN_ATOMS = x3, 0
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(3):
                    kernels.eq_scalar_head(x, v, head.output_network)
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()  # replayed: the kernels' time, not the host's
            with torch.cuda.graph(g):
                for _ in range(20):
                    kernels.eq_scalar_head(x, v, head.output_network)
            g.replay()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            torch.cuda.synchronize()
            ev[0].record()
            for _ in range(5):
                g.replay()
            ev[1].record()
            torch.cuda.synchronize()
            row["mfma" if x3 else "valu"] = round(1000 * ev[0].elapsed_time(ev[1]) / 100, 2)
        out[n] = row
    print(json.dumps(out))


if __name__ == "__main__":
    main()
