"""Fused dk/dv projection edge kernel (csrc/et_fused.hip) vs the unfused model layout (projection GEMM
over the pair rows + tmdnet_et_message_fwd reading them), on the C5 water box: outputs compared and
both timed with HIP events on the launch stream.

usage (GPU box, repo root): python tools/fep_time.py [n_atoms] [R]"""
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "torchmd-net_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def timed(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    from torchmdnet import kernels
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 50001
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    H, dev = 128, torch.device("cuda", 0)
    launch, E, L = bench.probe_workload(n, H, dev)
    g = launch.graph
    r = g.distances.detach()
    cl, cu = 0.0, 5.0
    alpha = 5.0 / (cu - cl)
    start = math.exp(-cu + cl)
    mu = torch.linspace(start, 1.0, R, device=dev)
    beta = torch.full((R,), (2.0 / R * (1 - start)) ** -2, device=dev)
    gen = torch.Generator(device=dev).manual_seed(11)
    W = torch.randn(4 * H, R, device=dev, generator=gen) / R ** 0.5
    b = torch.randn(4 * H, device=dev, generator=gen) * 0.1
    q, k, v, vec, C, u = launch.inputs
    if os.environ.get("FEP_TIME_QKV") == "strided":  # the model's layout: q | k | v views of one [N, 5H] buffer
        qkv = torch.cat([q, k, v], 1).contiguous()
        q, k, v = qkv[:, :H], qkv[:, H:2 * H], qkv[:, 2 * H:]
    # unfused: pair-row features -> projection GEMM -> message kernel over pair rows
    pair_row, pair_edge = launch.pair_row, launch.pair_edge
    f_pairs = kernels.rbf_composite(r.index_select(0, pair_edge.long()), mu, beta, cl, cu, 0).contiguous()
    xo0, vo0 = torch.empty(n, H, device=dev), torch.empty(n, 3, H, device=dev)
    xo1, vo1 = torch.empty(n, H, device=dev), torch.empty(n, 3, H, device=dev)
    wp = kernels.proj_split(W)

    def unfused_proj():
        return kernels.proj(f_pairs, W, b, wp=wp)

    pkv = unfused_proj()

    def unfused_msg():
        kernels.et_message_fwd_launch(q, k, v, vec, pkv[:, :H], pkv[:, H:], C, u, g, 8, xo0, vo0,
                                      flags=4, pk_rows=pair_row)

    fep = kernels.fep_split(W, b)
    frag = kernels.fep_frag_set(g, r, (mu, beta, cl, cu, 0), (pair_row, pair_edge))

    def fused():
        kernels.et_fused_fwd_launch(q, k, v, vec, C, u, fep, frag, g, 8, xo1, vo1, flags=4)

    if len(sys.argv) > 3 and sys.argv[3] == "fused_only":  # profiling: the fused launches alone
        for _ in range(10):
            fused()
        torch.cuda.synchronize()
        return
    if len(sys.argv) > 3 and sys.argv[3] == "fused_bwd_only":  # profiling: the fused backward alone
        gx_, gv_ = torch.randn(n, H, device=dev), torch.randn(n, 3, H, device=dev)
        bufs = [torch.empty(n, H, device=dev), torch.empty(n, H, device=dev), torch.empty(n, 3 * H, device=dev),
                torch.empty(n, 3, H, device=dev), torch.empty(E, device=dev), torch.empty(E, 3, device=dev),
                torch.empty(E, device=dev)]
        for _ in range(6):
            kernels.et_fused_bwd_launch(q, k, v, vec, C, u, fep, frag, g, 8, gx_, gv_, *bufs,
                                        accumulate=1 | 4)
        torch.cuda.synchronize()
        return
    unfused_msg()
    fused()
    torch.cuda.synchronize()
    rows_info = {}
    err_x = float((xo1 - xo0).abs().max() / xo0.abs().max())
    err_v = float((vo1 - vo0).abs().max() / vo0.abs().max())
    reps = 20
    t_proj = timed(unfused_proj, reps)
    t_msg = timed(unfused_msg, reps)
    t_fused = timed(fused, reps)
    # the force-pass backward (dr mode): unfused = d(dk,dv)/dr GEMM over the pair rows + the dst/src passes
    # reading both row sets; fused = tmdnet_et_fused_bwd_f32 (d pre / d r on the MFMA in-kernel)
    fdp = kernels.rbf_deriv(r, mu, beta, cl, cu, 0, rows=pair_edge)
    gen2 = torch.Generator(device=dev).manual_seed(5)
    gx, gvec = torch.randn(n, H, device=dev, generator=gen2), torch.randn(n, 3, H, device=dev, generator=gen2)
    def grads():  # gradient buffers with the row strides of q / k / v (the kernels write with them)
        gqkv = torch.empty(n, q.stride(0), device=dev)
        if q.stride(0) == H:  # separate contiguous q / k / v
            gq_, gk_, gv_ = torch.empty(n, H, device=dev), torch.empty(n, H, device=dev), \
                torch.empty(n, 3 * H, device=dev)
        else:  # views of one [N, 5H] buffer
            gq_, gk_, gv_ = gqkv[:, :H], gqkv[:, H:2 * H], gqkv[:, 2 * H:5 * H]
        return [gq_, gk_, gv_, torch.empty(n, 3, H, device=dev), torch.empty(E, device=dev),
                torch.empty(E, 3, device=dev), torch.empty(E, device=dev)]

    outs = [grads() for _ in range(3)]

    def unfused_dproj():
        return kernels.proj(fdp, W, None, wp=wp)

    dpkv = unfused_dproj()

    def unfused_bwd():
        gq, gk, gv, gw, gC, gu, gr = outs[0]
        kernels.et_message_bwd_launch(q, k, v, vec, pkv[:, :H], pkv[:, H:], C, u, g, 8, gx, gvec, gq, gk, gv, gw,
                                      None, None, gC, gu, accumulate=1 | 4, pk_rows=pair_row, dpk=dpkv[:, :H],
                                      dpv=dpkv[:, H:], g_r=gr)

    def unfused_bwd_2pass():  # the same call as the two passes (TMDNET_ET_TWO_PASS)
        gq, gk, gv, gw, gC, gu, gr = outs[2]
        kernels.et_message_bwd_launch(q, k, v, vec, pkv[:, :H], pkv[:, H:], C, u, g, 8, gx, gvec, gq, gk, gv, gw,
                                      None, None, gC, gu, accumulate=1 | 4 | 64, pk_rows=pair_row,
                                      dpk=dpkv[:, :H], dpv=dpkv[:, H:], g_r=gr)

    def fused_bwd():
        gq, gk, gv, gw, gC, gu, gr = outs[1]
        kernels.et_fused_bwd_launch(q, k, v, vec, C, u, fep, frag, g, 8, gx, gvec, gq, gk, gv,
                                    gw, gC, gu, gr, accumulate=1 | 4)

    unfused_bwd()
    fused_bwd()
    unfused_bwd_2pass()
    torch.cuda.synchronize()
    merged_err = {nm: float((b - a).abs().max() / a.abs().max()) for nm, a, b in
                  zip("gq gk gv gvec gC gu gr".split(), outs[2], outs[0])}
    bwd_err = {nm: float((b - a).abs().max() / a.abs().max()) for nm, a, b in
               zip("gq gk gv gvec gC gu gr".split(), outs[0], outs[1])}
    t_dproj = timed(unfused_dproj, reps)
    t_ubwd = timed(unfused_bwd, reps)
    t_fbwd = timed(fused_bwd, reps)
    t_u2 = timed(unfused_bwd_2pass, reps)
    flop = 2.0 * E * R * 4 * H
    out = {**rows_info, "n_atoms": n, "edges": E, "pairs": int(pair_edge.shape[0]), "R": R,
           "max_rel_err_x": err_x, "max_rel_err_vec": err_v,
           "unfused_proj_ms": round(t_proj, 4), "unfused_msg_ms": round(t_msg, 4),
           "unfused_total_ms": round(t_proj + t_msg, 4), "fused_ms": round(t_fused, 4),
           "fused_fp32_equiv_tflops": round(flop / t_fused / 1e9, 1),
           "fused_f16_mfma_tflops": round(3 * flop / t_fused / 1e9, 1),
           "bwd_max_rel_err": bwd_err, "unfused_dproj_ms": round(t_dproj, 4), "unfused_bwd_ms": round(t_ubwd, 4),
           "unfused_bwd_total_ms": round(t_dproj + t_ubwd, 4), "fused_bwd_ms": round(t_fbwd, 4),
           "two_pass_bwd_ms": round(t_u2, 4), "merged_vs_two_pass_err": merged_err}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
