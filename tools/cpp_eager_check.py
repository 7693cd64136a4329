"""Eval-mode eager C2 evaluation through the C++ tmdnet::et_stack operator vs the Python layer stack vs the
fp64 oracle (energies / forces, max-abs error over max |value|), and the eager time of each route.
usage (GPU box, repo root): python3 tools/cpp_eager_check.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "torchmd-net_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

import bench  # noqa: E402


def rel(a, b):
    return float((a.double().cpu() - b.double().cpu()).abs().max() / b.double().cpu().abs().max())


def main():
    from oracle import model_oracle as O
    from torchmdnet.models import torchmd_et
    from torchmdnet.models.model import create_model
    args = bench.et_args(128)
    torch.manual_seed(0)
    m = create_model(args)
    z, pos, batch = O.qm9_like(32)
    y_ref, f_ref = O.energy_forces(m.state_dict(), dict(args), z, pos, batch)
    m = m.to("cuda").eval()
    z, pos, batch = z.cuda(), pos.float().cuda(), batch.cuda()
    out = {}
    for cpp in (True, False):
        torchmd_et.CPP_EAGER = cpp
        y, f = m(z, pos, batch)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(50):
            m(z, pos, batch)
        torch.cuda.synchronize()
        out["cpp" if cpp else "python"] = {"ms": round(1000 * (time.perf_counter() - t0) / 50, 3),
                                           "e_rel": rel(y.detach(), y_ref.detach()), "f_rel": rel(f.detach(), f_ref),
                                           "y": y.detach().cpu(), "f": f.detach().cpu()}
    d = {k: {a: b for a, b in v.items() if a not in ("y", "f")} for k, v in out.items()}
    d["cpp_vs_python"] = {"e": rel(out["cpp"]["y"], out["python"]["y"]), "f": rel(out["cpp"]["f"], out["python"]["f"])}
    print(json.dumps(d))


if __name__ == "__main__":
    main()
