"""List GEMM calls (mm/addmm/addmm_) of a torch.profiler chrome trace with shapes and kernel time."""
import json
import sys
from collections import defaultdict

tr = json.load(open(sys.argv[1]))
ev = tr["traceEvents"] if isinstance(tr, dict) else tr
launch = {}
for e in ev:
    if e.get("cat") in ("cuda_runtime", "cuda_driver") and "args" in e and e["args"].get("correlation") is not None:
        launch[e["args"]["correlation"]] = e
ops = defaultdict(list)
for e in ev:
    if e.get("ph") == "X" and e.get("cat") == "cpu_op" and e["name"] in ("aten::mm", "aten::addmm", "aten::addmm_", "aten::bmm", "aten::baddbmm"):
        ops[(e["pid"], e["tid"])].append(e)
agg = defaultdict(lambda: [0, 0.0, ""])
for k in ev:
    if k.get("cat") != "kernel":
        continue
    L = launch.get(k["args"].get("correlation"))
    if L is None:
        continue
    encl = [e for e in ops[(L["pid"], L["tid"])] if e["ts"] <= L["ts"] <= e["ts"] + e["dur"]]
    if not encl:
        continue
    e = min(encl, key=lambda e: e["dur"])
    key = (e["name"], str(e["args"].get("Input Dims")))
    a = agg[key]
    a[0] += 1
    a[1] += k["dur"]
    a[2] = k["name"][:60]
tot = 0
for (name, dims), (n, t, kn) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    tot += t
    print(f"{t:7.1f} us {n:3d}  {t / n:5.1f} us/call  {name:12s} {dims[:70]:70s} {kn}")
print("total", round(tot, 1))
