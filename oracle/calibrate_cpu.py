"""ORACLE calibration -- test infrastructure, runs in the BUILD CONTAINER only (needs /root/reference).

SURVEY.md 8(d): the CPU baseline timed on the GPU box is this repo's restatement
(oracle/model_oracle.py), because the reference cannot travel.  This script times the restatement
and the reference itself (the shimmed copy of ``oracle/pyref/setup_ref.sh``, run in a child process
whose sys.path holds only that copy) side by side on the same host threads, the same inputs and
the same weights, and records the ratio (the survey's bar: within +-15 %).

    python oracle/calibrate_cpu.py [--threads 8] [--seconds 20] [--out profiles/r02_cpu_calibration.json]

Cases: C2 energy+forces (ET-QM9 128 ch, 32 QM9-like molecules), C2 training step (E+F MSE,
double backward, AdamW), C4 ET-SPICE energy+forces, C3 TensorNet-rMD17 energy+forces.  The
reference model is built with the reference create_model from the same args and loaded with this
repo's state_dict (the keys are identical), and run with derivative=True (model.py:286-298).
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

CHILD = r'''
import json, sys, time, torch
torch.set_num_threads(int(sys.argv[2]))
cfg = torch.load(sys.argv[1], weights_only=True)  # written by the parent process (this repo)
from torchmdnet.models.model import create_model
res = {}
for name, c in cfg["cases"].items():
    args = dict(c["args"])
    m = create_model(args)
    m.load_state_dict(c["sd"])
    z, pos, batch = c["z"], c["pos"].float(), c["batch"]
    if c["kind"] == "train":
        opt = torch.optim.AdamW(m.parameters(), lr=4e-4)
        y_lab, f_lab = c["y"], c["f"]
        def fn():
            opt.zero_grad()
            y, f = m(z, pos.clone(), batch)
            loss = torch.nn.functional.mse_loss(y, y_lab) + torch.nn.functional.mse_loss(f, f_lab)
            loss.backward()
            opt.step()
    else:
        def fn():
            m(z, pos.clone(), batch)
    fn()
    n, t0 = 0, time.perf_counter()
    while True:
        fn()
        n += 1
        el = time.perf_counter() - t0
        if el >= cfg["seconds"] or n >= 500:
            break
    res[name] = {"calls": n, "seconds": el, "ms_per_call": 1000 * el / n}
print(json.dumps(res))
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--seconds", type=float, default=8.0, help="per case, per side, per round")
    ap.add_argument("--rounds", type=int, default=3,
                    help="alternating restatement / reference rounds; the minimum per case is kept")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r02_cpu_calibration.json"))
    a = ap.parse_args()
    sys.path[:0] = [os.path.join(ROOT, "torchmd-net_amd"), ROOT]
    import torch
    import bench
    from oracle import model_oracle as O
    from torchmdnet.models.model import create_model
    import yaml

    torch.set_num_threads(a.threads)
    cases = {}

    def add(name, kind, args, n_mol, zpb, ref_args=None):
        torch.manual_seed(0)
        m = create_model(args)
        sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
        z, pos, batch = zpb
        gy = torch.Generator().manual_seed(100)
        cases[name] = {"kind": kind, "args": dict(ref_args or args), "sd": sd, "z": z, "pos": pos, "batch": batch,
                       "y": torch.randn(n_mol, 1, generator=gy), "f": torch.randn(z.shape[0], 3, generator=gy),
                       "oracle_args": dict(args), "pnames": sorted(k for k, _ in m.named_parameters())}

    et = bench.et_args(128)
    add("c2_energy_forces", "infer", et, 32, bench.qm9_like(32, 1))
    add("c2_train_step", "train", et, 32, bench.qm9_like(32, 1))
    add("c4_et_spice_energy_forces", "infer", bench.spice_model_args(), 16, bench.spice_like(16, 1))
    with open(os.path.join(ROOT, "tests", "golden", "configs", "tensornet_rmd17.yaml")) as f:
        targs = yaml.safe_load(f)
    targs.update(prior_model=None, precision=32, derivative=True)
    # the reference CPU op never pads, whatever static_shapes says: the
    # restatement runs its unpadded branch to match it
    add("c3_tensornet_rmd17_energy_forces", "infer", targs, 8, bench.rmd17_like(8, 1))

    fns = {}
    for name, c in cases.items():
        if c["kind"] == "train":
            leaf = {k: (v.clone().requires_grad_(True) if k in c["pnames"] else v) for k, v in c["sd"].items()}
            opt = torch.optim.AdamW([leaf[k] for k in c["pnames"]], lr=4e-4)

            def fn(c=c, leaf=leaf, opt=opt):
                opt.zero_grad()
                y, f = O.energy_forces(leaf, c["oracle_args"], c["z"], c["pos"].float(), c["batch"],
                                       dtype=torch.float32, create_graph=True)
                loss = torch.nn.functional.mse_loss(y, c["y"]) + torch.nn.functional.mse_loss(f, c["f"])
                loss.backward()
                opt.step()
        else:
            def fn(c=c):
                O.energy_forces(c["sd"], c["oracle_args"], c["z"], c["pos"].float(), c["batch"],
                                dtype=torch.float32, static_shapes=False, create_graph=True)
        fns[name] = fn

    def time_restatement():
        out = {}
        for name, fn in fns.items():
            fn()
            n, t0 = 0, time.perf_counter()
            while True:
                fn()
                n += 1
                el = time.perf_counter() - t0
                if el >= a.seconds or n >= 500:
                    break
            out[name] = 1000 * el / n
        return out

    ref_dir = subprocess.check_output(["bash", os.path.join(HERE, "pyref", "setup_ref.sh")], text=True).strip()
    mine, ref = {k: [] for k in cases}, {k: [] for k in cases}
    with tempfile.TemporaryDirectory() as td:
        cfg_path = os.path.join(td, "cases.pt")
        torch.save({"cases": {k: {kk: vv for kk, vv in v.items() if kk not in ("oracle_args", "pnames")}
                              for k, v in cases.items()}, "seconds": a.seconds}, cfg_path)
        child = os.path.join(td, "child.py")
        open(child, "w").write(CHILD)
        env = {k: v for k, v in os.environ.items() if k != "PYTHONPATH"}
        env.update(PYTHONPATH=f"{ref_dir}/shims:{ref_dir}", TORCH_EXTENSIONS_DIR=f"{ref_dir}/torch_ext")
        for rnd in range(a.rounds):
            for k, v in time_restatement().items():
                mine[k].append(v)
            # the reference, in a child process that sees only the shimmed copy
            out = subprocess.check_output([sys.executable, child, cfg_path, str(a.threads)], env=env, cwd=td,
                                          text=True, stderr=subprocess.DEVNULL)
            for k, v in json.loads(out.strip().splitlines()[-1]).items():
                ref[k].append(v["ms_per_call"])
            print("round", rnd, {k: (round(mine[k][-1], 1), round(ref[k][-1], 1)) for k in cases}, flush=True)

    res = {"what": "CPU restatement (oracle/model_oracle.py, timed on the GPU box as cpu_baseline) vs the shimmed "
                   "reference (oracle/pyref/setup_ref.sh), same inputs / weights / threads, float32, "
                   "derivative=True",
           "host": bench.host_cpu_info(), "threads": a.threads, "seconds_per_case_round": a.seconds,
           "rounds": a.rounds, "statistic": "minimum over the alternating rounds (per side)",
           "bar": "ratio restatement_ms / reference_ms within 0.85 .. 1.15 (SURVEY.md 8(d))", "cases": {}}
    for name in cases:
        mm, rr = min(mine[name]), min(ref[name])
        r = mm / rr
        res["cases"][name] = {"restatement_ms": round(mm, 2), "reference_ms": round(rr, 2),
                              "restatement_rounds_ms": [round(v, 1) for v in mine[name]],
                              "reference_rounds_ms": [round(v, 1) for v in ref[name]],
                              "ratio": round(r, 3), "within_15pct": abs(r - 1) <= 0.15}
        print(name, res["cases"][name], flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print("wrote", a.out)


if __name__ == "__main__":
    main()
