"""Attribute GPU kernels matching a name/grid to the ATen op and Python frames that launched them,
from a torch.profiler chrome trace (diagnosis).  usage: kernel_owner.py trace.json NAME [GRIDX]"""
import json
import sys

tr = json.load(open(sys.argv[1]))
ev = tr["traceEvents"] if isinstance(tr, dict) else tr
name = sys.argv[2]
gridx = int(sys.argv[3]) if len(sys.argv) > 3 else None
launch = {}
for e in ev:
    if e.get("cat") in ("cuda_runtime", "cuda_driver") and "args" in e:
        c = e["args"].get("correlation")
        if c is not None:
            launch[c] = e
spans = [e for e in ev if e.get("ph") == "X" and e.get("cat") in ("cpu_op", "python_function", "user_annotation")]
by_tid = {}
for e in spans:
    by_tid.setdefault((e["pid"], e["tid"]), []).append(e)
seen = 0
for k in ev:
    if k.get("cat") != "kernel" or name not in k.get("name", ""):
        continue
    g = k["args"].get("grid", [0])
    if gridx is not None and g[0] != gridx:
        continue
    L = launch.get(k["args"].get("correlation"))
    if L is None:
        print("kernel without launch", g)
        continue
    t = L["ts"]
    encl = [e for e in by_tid.get((L["pid"], L["tid"]), []) if e["ts"] <= t <= e["ts"] + e["dur"]]
    encl.sort(key=lambda e: e["dur"])
    print("=== kernel grid", g, k["args"].get("block"))
    for e in encl[:14]:
        a = e.get("args", {})
        print("   ", e["cat"][:6], e["name"][:100], a.get("Input Dims", ""))
    seen += 1
    if seen >= 4:
        break
print("matches:", seen)
