"""Isolated timing of the x3 GEMM (kernels.gemm_ex_launch above GEMM_MAX_ROWS -> tmdnet_gemm_x3_ex_f32) at the
C5 TensorNet shapes: the pair-row edge MLP (P ~ 1.0M rows: 32 -> 128 -> 256 -> 384 with the SiLU / pre /
cutoff epilogues; the backward's input gradients with the silu' epilogue) and the embedding's distance
projection over the edges (E ~ 1.96M, 32 -> 384).  us per call, bytes (A + epilogue operands + outputs) / time,
bf16 TFLOP/s of the six split products.  usage: python tools/x3_tn_time.py   (TMDNET_X3_BN=64|128 A/B)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "torchmd-net_amd"), ROOT]
import torch  # noqa: E402

from torchmdnet import kernels  # noqa: E402

dev = torch.device("cuda", 0)


def timed(fn, reps=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    P, E = 1005552, 1961103
    g = torch.Generator(device=dev).manual_seed(0)
    shapes = [("L1_fwd", P, 128, 32, "act"), ("L2_fwd", P, 256, 128, "act"), ("L3_fwd", P, 384, 256, "act_scale"),
              ("L3_bwd", P, 256, 384, "dpre"), ("L2_bwd", P, 128, 256, "dpre"), ("L1_bwd", P, 32, 128, "none_t"),
              ("dist_proj", E, 384, 32, "bias")]
    for name, M, N, K, mode in shapes:
        A = torch.randn(M, K, device=dev, generator=g)
        tb = not mode.endswith("_t") and mode != "dpre"
        W = torch.randn(N, K, device=dev, generator=g) / K ** 0.5 if tb else torch.randn(K, N, device=dev, generator=g)
        C = torch.empty(M, N, device=dev)
        p = {"A": A, "B": W, "trans_b": tb, "C": C}
        nb = 4 * (M * K + M * N)
        if mode.startswith("act"):
            p.update(bias=torch.randn(N, device=dev, generator=g), pre=torch.empty(M, N, device=dev), act=1)
            nb += 4 * M * N
            if mode == "act_scale":
                p["rscale"] = torch.rand(M, device=dev, generator=g)
        elif mode == "dpre":
            p["dpre"] = torch.randn(M, N, device=dev, generator=g)
            nb += 4 * M * N
        elif mode == "bias":
            p["bias"] = torch.randn(N, device=dev, generator=g)
        assert kernels.gemm_ex_launch([p])
        t = timed(lambda: kernels.gemm_ex_launch([p]))
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "us": round(t, 1), "TBps": round(nb / t / 1e6, 2),
                          "bf16_TFs": round(12 * M * N * K / t / 1e6, 1)}), flush=True)
        del A, W, C, p


if __name__ == "__main__":
    main()
