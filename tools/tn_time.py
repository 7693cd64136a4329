"""HIP-event timing of the grouped weight-gradient TN GEMM (kernels.wgrad_tn) on the training step's shapes,
for each kernel form (TMDNET_TN_V=1: k_gemm_tn_v, 2: the pipelined k_gemm_tn_v2).
usage (GPU box, repo root): python tools/tn_time.py > gpurun_out/tn_time.txt"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "torchmd-net_amd"), ROOT]
import torch  # noqa: E402

from bench import qm9_like  # noqa: E402
from torchmdnet import kernels  # noqa: E402

dev = torch.device("cuda", 0)
z, pos, batch = qm9_like(32, 1)
pos, batch = pos.float().to(dev), batch.to(dev)
same = batch[:, None] == batch[None, :]
r = torch.cdist(pos, pos)
n_atoms = z.shape[0]
pairs = int(((r < 5.0) & same).triu(1).sum())
Ep = n_atoms + pairs  # pair rows (self loops + one row per unordered pair)
H, L, R = 128, 8, 64  # (et_qm9.yaml: num_rbf 64)
print(f"atoms {n_atoms} pairs {pairs} pair rows {Ep}")


def dkv_probs(k2):
    A = torch.randn(Ep, L * 4 * H, device=dev)
    B = torch.randn(Ep, R, device=dev)
    p = {"A": A, "B": B, "C": torch.empty(L * 4 * H, R, device=dev), "Cb": torch.empty(L * 4 * H, device=dev),
         "ones": True}
    if k2:
        p.update(A2=torch.randn(k2, L * 4 * H, device=dev), B2=torch.randn(k2, R, device=dev), ones2=False)
    return [p]


def node_probs():
    N = n_atoms
    probs = []
    for l in range(L):
        def seg(m, n, rows):
            return {"A2": torch.randn(rows, m, device=dev), "B2": torch.randn(rows, n, device=dev)}
        probs.append({"A": torch.randn(N, 3 * H, device=dev), "B": torch.randn(N, H, device=dev),
                      "C": torch.empty(3 * H, H, device=dev), "Cb": torch.empty(3 * H, device=dev), "ones": True,
                      **seg(3 * H, H, N)})
        probs.append({"A": torch.randn(N, 3 * H, device=dev), "B": torch.randn(N, H, device=dev),
                      "C": torch.empty(3 * H, H, device=dev), "Cb": torch.empty(3 * H, device=dev), "ones": True,
                      **seg(3 * H, H, N)})
        if l:
            probs.append({"A": torch.randn(3 * N, 3 * H, device=dev), "B": torch.randn(3 * N, H, device=dev),
                          "C": torch.empty(3 * H, H, device=dev), **seg(3 * H, H, 3 * N)})
        probs.append({"A": torch.randn(N, H, device=dev), "B": None, "C": torch.empty(H, 1, device=dev),
                      "ones": True, "A2": torch.randn(N, H, device=dev), "ones2": True})
        probs.append({"A": torch.randn(N, H, device=dev), "B": None, "C": torch.empty(H, 1, device=dev),
                      "ones": True})
    return probs


def timed(probs, reps=50):
    for _ in range(5):
        kernels.wgrad_tn(probs)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        kernels.wgrad_tn(probs)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


cases = [("dkv K2=Ep", dkv_probs(Ep)), ("dkv K2=2Ep", dkv_probs(2 * Ep)), ("node x8 layers", node_probs())]
for name, probs in cases:
    for target in ("1024", "2048"):
        os.environ["TMDNET_TN_TARGET"] = target
        row = []
        for form in ("1", "2", "3", "4", "5"):
            os.environ["TMDNET_TN_V"] = form
            row.append(timed(probs))
        print(f"{name:16s} target {target:5s} form1 {row[0]:7.1f} us  form2 (pipelined) {row[1]:7.1f} us  form3 {row[2]:7.1f} us  "
              f"form4 (bf16x3) {row[3]:7.1f} us  form5 (bf16x3 regs) {row[4]:7.1f} us", flush=True)
