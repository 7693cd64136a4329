import sys, os, torch
sys.path.insert(0, 'tests'); sys.path.insert(0, 'torchmd-net_amd'); sys.path.insert(0, '.')
import test_gpu_fused as T
from torchmdnet import et_stack, kernels
z, pos, L = T._water_box(3000)
m = T._model(64, "expnorm", 0.0)
cap = {}
orig = kernels.et_message_bwd_launch
def bw(*a, **k):
    d = cap.setdefault(et_stack.FEP, [])
    names = "q k v vec pk pv C u graph heads gx gvec gq gk gv gw gpk gpv gC gu".split()
    ent = {n: (x.clone() if torch.is_tensor(x) else x) for n, x in zip(names, a)}
    for kk in ("dpk", "dpv", "pk_rows"):
        ent[kk] = k.get(kk).clone() if torch.is_tensor(k.get(kk)) else k.get(kk)
    ent["acc"] = k.get("accumulate")
    g_r = k.get("g_r")
    ent["gr_before"] = g_r.clone()
    orig(*a, **k)
    ent["gr_after"] = g_r.clone()
    d.append(ent)
kernels.et_message_bwd_launch = bw
for fep in ("auto", "0"):
    et_stack.FEP = fep
    T._run(m, z, pos, L, torch.float32)
A, B = cap["auto"], cap["0"]
def rel(x, y):
    if x is None or y is None: return (x is None, y is None)
    if not torch.is_tensor(x): return x == y
    return float((x.double() - y.double()).abs().max() / y.double().abs().max().clamp_min(1e-30))
for i, (a, b) in enumerate(zip(A, B)):
    print(i, {k: rel(a[k], b[k]) for k in a if k not in ("graph",)})
    print("  gr_before finite", bool(torch.isfinite(a["gr_before"]).all()), "E", a["gr_before"].shape)
