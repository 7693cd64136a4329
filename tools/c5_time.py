"""C5 water box (50,001 atoms, ET 128 ch x 8 layers, cutoff 5, periodic, cell list) energy + forces,
timed eagerly as bench.py's secondary_water_box does; the edge-kernel variant comes from the
environment (TMDNET_FEP, TMDNET_FEP_BWD).  usage: python tools/c5_time.py [n_atoms] [steps] [script]"""
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
    from torchmdnet.models.model import create_model
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 50001
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    dev = torch.device("cuda", 0)
    args = bench.et_args(128)
    args.update(max_num_neighbors=128)
    torch.manual_seed(0)
    model = create_model(args).to(dev)
    g = torch.Generator().manual_seed(7)
    L = (n / 0.1003) ** (1.0 / 3.0)
    pos = (torch.rand(n, 3, generator=g, dtype=torch.float64) * L).float().to(dev)
    z = torch.tensor([8, 1, 1], dtype=torch.long).repeat(n // 3 + 1)[:n].to(dev)
    batch = torch.zeros(n, dtype=torch.long, device=dev)
    d = model.representation_model.distance
    d.box = torch.eye(3, dtype=torch.float32) * L
    d.use_periodic = True
    d.strategy = "cell"
    if len(sys.argv) > 3 and sys.argv[3] == "script":  # the MD-engine form: one tmdnet::et_energy_forces
        model = torch.jit.script(model.eval())
    for _ in range(2):
        y, f = model(z, pos, batch)
    torch.cuda.synchronize()
    m0 = torch.cuda.memory_stats()
    t0 = time.perf_counter()
    host = 0.0
    for _ in range(steps):
        h0 = time.perf_counter()
        y, f = model(z, pos, batch)
        host += time.perf_counter() - h0  # host time to enqueue (the queue may back up: an upper bound)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / steps
    m1 = torch.cuda.memory_stats()
    mem = {k: m1.get(k, 0) - m0.get(k, 0) for k in ("num_device_alloc", "num_device_free", "num_alloc_retries")}
    mem["peak_gb"] = round(torch.cuda.max_memory_allocated() / 2 ** 30, 1)
    mem["host_ms_per_eval"] = round(1000 * host / steps, 2)
    print(json.dumps({"fep": os.environ.get("TMDNET_FEP", "auto"), "fep_bwd": os.environ.get("TMDNET_FEP_BWD", "off"),
                      "ms_per_eval": round(1000 * el, 2), "atoms_per_s": round(n / el, 1),
                      "energy": float(y.detach().sum()), "force_absmax": float(f.abs().max()),
                      "force_sum": [float(v) for v in f.double().sum(0)], **mem}))


if __name__ == "__main__":
    main()
