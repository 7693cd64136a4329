"""Same-process A/B of the eval-mode eager C2 evaluation (host-bound, so boxes differ by tens of percent):
the Python layer stack, the C++ et_stack route (torchmd_et.CPP_EAGER), and the C++ route without the early
molecule-count read-back (TorchMD_Net._early_dim_size), interleaved rounds, ms per evaluation.
usage (GPU box, repo root): python3 tools/eager_ab.py [rounds]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "torchmd-net_amd")]
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    from torchmdnet.models import torchmd_et
    from torchmdnet.models.model import TorchMD_Net, create_model
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = create_model(bench.et_args(128)).to(dev).eval()
    z, pos, batch = bench.qm9_like(32, gen_seed=1)
    z, pos, batch = z.to(dev), pos.float().to(dev), batch.to(dev)
    early = TorchMD_Net._early_dim_size
    forms = {"python_stack": (False, early), "cpp_stack": (True, early),
             "cpp_stack_late_readback": (True, lambda self, b: None)}
    res = {k: [] for k in forms}
    for _ in range(rounds):
        for name, (cpp, hook) in forms.items():
            torchmd_et.CPP_EAGER = cpp
            TorchMD_Net._early_dim_size = hook
            for _ in range(5):
                m(z, pos, batch)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(40):
                m(z, pos, batch)
            torch.cuda.synchronize()
            res[name].append(1000 * (time.perf_counter() - t0) / 40)
    TorchMD_Net._early_dim_size = early
    print(json.dumps({k: {"median_ms": round(sorted(v)[len(v) // 2], 3), "all": [round(x, 3) for x in v]}
                      for k, v in res.items()}))


if __name__ == "__main__":
    main()
