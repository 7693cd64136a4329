"""Aggregate GPU kernel time of a torch.profiler chrome trace by the innermost torchmdnet Python
frame (file:line) that launched it (diagnosis).  usage: kernel_sites.py trace.json [top]"""
import json
import sys
from collections import defaultdict

tr = json.load(open(sys.argv[1]))
ev = tr["traceEvents"] if isinstance(tr, dict) else tr
top = int(sys.argv[2]) if len(sys.argv) > 2 else 60
launch = {}
for e in ev:
    if e.get("cat") in ("cuda_runtime", "cuda_driver") and "args" in e and e["args"].get("correlation") is not None:
        launch[e["args"]["correlation"]] = e
spans = defaultdict(list)
for e in ev:
    if e.get("ph") == "X" and e.get("cat") in ("cpu_op", "python_function"):
        spans[(e["pid"], e["tid"])].append(e)
agg = defaultdict(lambda: [0, 0.0, set()])
tot = 0.0
for k in ev:
    if k.get("cat") != "kernel":
        continue
    L = launch.get(k["args"].get("correlation"))
    site = "?"
    if L is not None:
        encl = [e for e in spans[(L["pid"], L["tid"])] if e["ts"] <= L["ts"] <= e["ts"] + e["dur"]]
        encl.sort(key=lambda e: e["dur"])
        py = [e["name"] for e in encl if e["cat"] == "python_function" and "torchmdnet" in e["name"]]
        ops = [e["name"] for e in encl if e["cat"] == "cpu_op"]
        site = (py[0] if py else "(no torchmdnet frame)") + " | " + (ops[0] if ops else "")
    a = agg[site]
    a[0] += 1
    a[1] += k["dur"]
    a[2].add(k["name"][:40])
    tot += k["dur"]
print(f"kernels total {tot:.0f} us")
for s, (n, t, names) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"{t:8.1f} us {n:4d}  {s[:150]}")
