"""C5 TensorNet arm: TensorNet-rMD17's architecture (128 ch, 2 layers, 32 RBF, cutoff 4.5, O(3)) on a
periodic ~50k-atom water box (cell list), energy + forces, eager -- the model reference
benchmarks/inference.py:63-71 times (its systems are PDB files; here the SURVEY §8(d) water box).
usage: python tools/tn_c5_time.py [n_atoms] [steps] [static 0|1] [script]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "torchmd-net_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 50001
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    static = (sys.argv[3] != "0") if len(sys.argv) > 3 else True
    script = len(sys.argv) > 4 and sys.argv[4] == "script"
    dev = torch.device("cuda", 0)
    model, z, pos, batch, L = bench.tn_water_box_model(n, static, 0, dev)
    if script:
        model = torch.jit.script(model.eval())
    t_first = time.perf_counter()
    y, f = model(z, pos, batch)
    torch.cuda.synchronize()
    t_first = time.perf_counter() - t_first
    y, f = model(z, pos, batch)
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats()
    t0 = time.perf_counter()
    host = 0.0
    for _ in range(steps):
        h0 = time.perf_counter()
        y, f = model(z, pos, batch)
        host += time.perf_counter() - h0
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / steps
    d = model.representation_model.distance if not script else None
    print(json.dumps({"static_shapes": static, "script": script, "n": n, "ms_per_eval": round(1000 * el, 2),
                      "atoms_per_s": round(n / el, 1), "first_call_s": round(t_first, 2),
                      "host_ms_per_eval": round(1000 * host / steps, 2),
                      "edges": None if d is None else int(d.last_num_pairs),
                      "energy": float(y.detach().sum()), "force_absmax": float(f.abs().max()),
                      "force_sum": [float(v) for v in f.double().sum(0)],
                      "peak_gb": round(torch.cuda.max_memory_allocated() / 2 ** 30, 2)}))


if __name__ == "__main__":
    main()
