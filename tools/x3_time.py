"""Isolated timing of tmdnet_gemm_x3_f32 (kernels.gemm_x3: the node feature mixes of C5-size systems) at
the C5 evaluation's shapes (50,001 atoms, H = 128: the q|k|v and o / vec projections and their input
gradients), HIP events on the launch stream; the library fp32 GEMM beside it, and the error of both
against fp64.  Per shape: us per call, algorithmic bytes (A read once, C written, + C read with beta) /
time, bf16-MFMA TFLOP/s of the six split products.
usage (GPU box, repo root): python tools/x3_time.py   (TMDNET_X3_REMAP=0: the 2-D grid, A/B)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "torchmd-net_amd"), ROOT]
import torch  # noqa: E402

from torchmdnet import kernels  # noqa: E402

dev = torch.device("cuda", 0)


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    n = 50001
    shapes = [("qkv_fwd", n, 640, 128, 0), ("o_fwd", n, 384, 128, 0), ("vec_fwd", 3 * n, 384, 128, 0),
              ("o_bwd", n, 128, 384, 0), ("vec_bwd", 3 * n, 128, 384, 0), ("qkv_bwd", n, 128, 640, 1)]
    g = torch.Generator(device=dev).manual_seed(0)
    for name, M, N, K, beta in shapes:
        A = torch.randn(M, K, device=dev, generator=g)
        W = torch.randn(N, K, device=dev, generator=g) / K ** 0.5
        bias = torch.randn(N, device=dev, generator=g)
        C = torch.zeros(M, N, device=dev)
        C0 = torch.randn(M, N, device=dev, generator=g)
        ref = A.double() @ W.double().t() + bias.double() + (C0.double() if beta else 0)

        def x3():
            if beta:
                C.copy_(C0)
            assert kernels.gemm_x3(A, W, True, bias, C, beta)

        x3()
        err = float((C.double() - ref).abs().max() / ref.abs().max())

        def lib():
            if beta:
                torch.addmm(C0 + bias, A, W.t(), out=C)
            else:
                torch.addmm(bias, A, W.t(), out=C)

        lib()
        err_lib = float((C.double() - ref).abs().max() / ref.abs().max())
        cp = timed(lambda: C.copy_(C0)) if beta else 0.0
        t = timed(x3) - cp
        tl = timed(lib)
        byts = 4 * (M * K + M * N * (2 if beta else 1))
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "beta": beta, "x3_us": round(t, 1),
                          "x3_TBps": round(byts / t / 1e6, 2), "x3_bf16_TFs": round(12 * M * N * K / t / 1e6, 1),
                          "lib_us": round(tl, 1), "err_x3": err, "err_lib": err_lib}), flush=True)
        del A, C, C0, ref


if __name__ == "__main__":
    main()
