"""Diagnose a C++ et_stack (CPP_EAGER) vs Python-stack difference on the fit test's data: eval-mode energies
and forces of the fit test's model on its molecules, fresh and after an LNNP validation-style call.
usage (GPU box, repo root): python3 tools/cpp_eager_diag.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "torchmd-net_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

from conftest import yaml_args  # noqa: E402


def rel(a, b):
    return float((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30))


def main():
    from test_gpu_fit_graphed import _dataset
    from torchmdnet.data import collate
    from torchmdnet.models import torchmd_et
    from torchmdnet.models.model import create_model
    torch.manual_seed(0)
    args = yaml_args("equivariant-transformer", embedding_dimension=64, num_layers=2, num_rbf=32, num_heads=8,
                     derivative=True)
    m = create_model(args).cuda().eval()
    data = _dataset(80, seed=7)
    out = []
    for i in range(0, 80, 16):
        b = collate(data[i:i + 16])
        z, pos, batch = b.z.cuda(), b.pos.cuda(), b.batch.cuda()
        res = {}
        for cpp in (True, False):
            torchmd_et.CPP_EAGER = cpp
            with torch.set_grad_enabled(True):
                y, f = m(z, pos, batch)
            res[cpp] = (y.detach(), f.detach())
        g = m.representation_model.distance.graph(pos, batch)
        out.append({"batch": i, "E": int(g.n_edges), "symmetric": bool(g.symmetric),
                    "e": rel(res[True][0], res[False][0]), "f": rel(res[True][1], res[False][1])})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
