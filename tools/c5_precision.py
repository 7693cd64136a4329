"""fp32 error of the C5 water-box evaluation (ET 128 ch x 8 layers, 64 RBF, cutoff 5, periodic) against the
same weights in fp64, per large-system launch form: the fused-projection kernels (et_fused.hip) or the
pair-row path, node mixes on tmdnet_gemm_x3_f32 or the library GEMM.  Prints one JSON line per form:
energy relative error, force max-abs / max |F| and RMS relative error, and the worst atom.
usage: python tools/c5_precision.py [n_atoms] [layers]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "torchmd-net_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    from torchmdnet import et_stack, kernels
    from torchmdnet.models.model import create_model
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 50001
    layers = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    dev = torch.device("cuda", 0)
    args = bench.et_args(128)
    args.update(max_num_neighbors=128, num_layers=layers)
    torch.manual_seed(0)
    m32 = create_model(args).to(dev)
    a64 = dict(args, precision=64)
    m64 = create_model(a64).to(dev)
    m64.load_state_dict({k: v.double() if v.is_floating_point() else v for k, v in m32.state_dict().items()})
    g = torch.Generator().manual_seed(7)
    L = (n / 0.1003) ** (1.0 / 3.0)
    pos = (torch.rand(n, 3, generator=g, dtype=torch.float64) * L).to(dev)
    z = torch.tensor([8, 1, 1], dtype=torch.long).repeat(n // 3 + 1)[:n].to(dev)
    batch = torch.zeros(n, dtype=torch.long, device=dev)
    for m, dt in ((m32, torch.float32), (m64, torch.float64)):
        d = m.representation_model.distance
        d.box = torch.eye(3, dtype=dt) * L
        d.use_periodic = True
        d.strategy = "cell"
    y64x, f64x = m64(z, pos, batch)  # exact positions
    y64x, f64x = y64x.detach(), f64x.detach()
    # the reference on the fp32-rounded positions the fp32 model sees (input quantisation: ~5e-6 A at
    # L = 79 A, i.e. ~5e-5 relative on the delta of a 0.1 A pair)
    pos = pos.float().double()
    y64, f64 = m64(z, pos, batch)
    y64, f64 = y64.detach(), f64.detach()
    print(json.dumps({"rounding_only": {"energy_rel": float((y64 - y64x).abs().sum() / y64x.abs().sum()),
                                        "force_maxabs_rel": float((f64 - f64x).abs().max() / f64x.abs().max())}}),
          flush=True)
    del m64
    torch.cuda.empty_cache()
    fmax = f64.abs().max()
    for fep, big in (("auto", "x3"), ("auto", "lib"), ("0", "lib"), ("0", "x3")):
        et_stack.FEP = fep
        kernels.GEMM_BIG = big
        y, f = m32(z, pos.float(), batch)
        y, f = y.detach().double(), f.detach().double()
        err = (f - f64).abs()
        w = int(err.max(1).values.argmax())
        print(json.dumps({"fep": fep, "gemm_big": big, "n": n, "layers": layers,
                          "energy_rel": float((y - y64).abs().sum() / y64.abs().sum()),
                          "force_maxabs_rel": float(err.max() / fmax),
                          "force_rms_rel": float(err.pow(2).mean().sqrt() / f64.pow(2).mean().sqrt()),
                          "worst_atom": w, "worst_f64": [float(v) for v in f64[w]],
                          "worst_err": [float(v) for v in err[w]],
                          "fsum32": [float(v) for v in f.sum(0)]}), flush=True)


if __name__ == "__main__":
    main()
