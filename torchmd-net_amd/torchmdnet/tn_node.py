"""TensorNet node-level tensor algebra through the fused HIP passes of ``csrc/tn_node.hip``.

Reference: ``torchmdnet/models/tensornet.py`` -- ``decompose_tensor`` / ``tensor_norm`` (:47-67),
``TensorNet.forward``'s output norms (:230-231), ``TensorEmbedding.forward`` (:316-326) and
``Interaction.forward`` (:391-410).  The reference evaluates these as chains of elementwise
PyTorch kernels on ``[N, H, 3, 3]`` tensors (about 200 launches per TensorNet layer pair at
rMD17 size); here every step is one pass with a thread per (atom, channel).

Interior tensors use the COMPACT component-major layout ``[9, N, H]``: per channel the coefficients
``[i, a01, a02, a12, s00, s11, s01, s02, s12]`` of ``X = i*Id + A + S`` (rows 0 / 1-3 / 4-8 = the
I / A / S parts).  The reference's channel mixes ``linear(I.permute(0, 2, 3, 1))`` are then three
plain GEMMs over row blocks of one buffer (``mix3``), and the message kernel gathers 9 instead of
27 values per channel.

Every op is an autograd Function with HIP forward and HIP first backward; the backward is itself a
Function whose backward (second order, force-loss training only) differentiates the PyTorch
composite below twice -- the same scheme as the other hot-path ops (``kernels.py``).
"""
import os

import torch
from torch.autograd import Function

from . import _native as nat
from . import kernels

PRE, POST_O3, POST_SO3, RESID, NORMS, ENORM, EOUT = range(7)


# ----------------------------------------------------------------------------- composites
def full9(c):
    """compact (9, N, H) -> full (N, H, 3, 3)."""
    i, a01, a02, a12, s00, s11, s01, s02, s12 = c.unbind(0)
    F = torch.stack((i + s00, a01 + s01, a02 + s02,
                     s01 - a01, i + s11, a12 + s12,
                     s02 - a02, s12 - a12, i - s00 - s11), dim=-1)
    return F.view(*F.shape[:-1], 3, 3)


def decomp9(X):
    """full (N, H, 3, 3) -> compact (9, N, H): reference decompose_tensor (tensornet.py:47-52)."""
    f = X.reshape(*X.shape[:-2], 9).unbind(-1)
    i = (f[0] + f[4] + f[8]) / 3
    return torch.stack((i, 0.5 * (f[1] - f[3]), 0.5 * (f[2] - f[6]), 0.5 * (f[5] - f[7]),
                        f[0] - i, f[4] - i, 0.5 * (f[1] + f[3]), 0.5 * (f[2] + f[6]),
                        0.5 * (f[5] + f[7])), dim=0)


def _mm33(a, b):
    return (a.unsqueeze(-1) * b.unsqueeze(-3)).sum(-2)


def _tnorm(t):
    return (t ** 2).sum((-2, -1))


def op_composite(op, a, b=None):
    """PyTorch restatement of each fused pass (same layouts as the HIP op)."""
    if op == PRE:
        return decomp9(a / (_tnorm(a) + 1)[..., None, None])
    if op in (POST_O3, POST_SO3):
        Y, M = full9(a), full9(b)
        Z = _mm33(M, Y) + _mm33(Y, M) if op == POST_O3 else 2 * _mm33(Y, M)
        return decomp9(Z) / (_tnorm(Z) + 1)
    if op == RESID:  # the residual is the normalised input (the reference reassigns X, :391)
        D = full9(b)
        return a / (_tnorm(a) + 1)[..., None, None] + D + _mm33(D, D)
    if op == NORMS:
        c = decomp9(a)
        nI = 3 * c[0] ** 2
        nA = 2 * (c[1] ** 2 + c[2] ** 2 + c[3] ** 2)
        nS = c[4] ** 2 + c[5] ** 2 + (c[4] + c[5]) ** 2 + 2 * (c[6] ** 2 + c[7] ** 2 + c[8] ** 2)
        return torch.cat((nI, nA, nS), dim=-1)
    if op == ENORM:
        return _tnorm(full9(a))
    if op == EOUT:
        f = b.view(b.shape[0], -1, 3)
        scale = torch.stack([f[..., 0]] + [f[..., 1]] * 3 + [f[..., 2]] * 5, dim=0)
        return full9(a * scale)
    raise ValueError(op)


def _out_shape(op, a):
    if op == PRE:
        return (9, a.shape[0], a.shape[1])
    if op in (POST_O3, POST_SO3, RESID):
        return a.shape
    if op == NORMS:
        return (a.shape[0], 3 * a.shape[1])
    if op == ENORM:
        return (a.shape[1], a.shape[2])
    if op == EOUT:
        return (a.shape[1], a.shape[2], 3, 3)
    raise ValueError(op)


def _nh(op, a):
    """(N, H) of an op from its first input."""
    if op in (PRE, RESID, NORMS):
        return a.shape[0], a.shape[1]
    return a.shape[1], a.shape[2]


# ----------------------------------------------------------------------------- launches
def node_fwd_launch(op, a, b, out):
    lib = nat.load()
    n, h = _nh(op, a)
    rc = lib.tmdnet_tn_node_fwd(nat.dtype_code(a.dtype), op, n, h, nat.ptr(a), nat.ptr(b), nat.ptr(out),
                                nat.stream(a.device))
    nat.check(rc, f"tmdnet_tn_node_fwd(op={op})")


def node_bwd_launch(op, a, b, gout, gadd, ga, gb):
    lib = nat.load()
    n, h = _nh(op, a)
    rc = lib.tmdnet_tn_node_bwd(nat.dtype_code(a.dtype), op, n, h, nat.ptr(a), nat.ptr(b), nat.ptr(gout),
                                nat.ptr(gadd), nat.ptr(ga), nat.ptr(gb), nat.stream(a.device))
    nat.check(rc, f"tmdnet_tn_node_bwd(op={op})")


def node_bwd2_launch(op, a, b, gout, ta, tb, d_g, d_a, d_b):
    lib = nat.load()
    n, h = _nh(op, a)
    rc = lib.tmdnet_tn_node_bwd2(nat.dtype_code(a.dtype), op, n, h, nat.ptr(a), nat.ptr(b), nat.ptr(gout),
                                 nat.ptr(ta), nat.ptr(tb), nat.ptr(d_g), nat.ptr(d_a), nat.ptr(d_b),
                                 nat.stream(a.device))
    nat.check(rc, f"tmdnet_tn_node_bwd2(op={op})")


# the hand-written second orders (tmdnet_tn_node_bwd2, the channel mixes' GEMMs); "composite": autograd's
# double differentiation of the PyTorch restatements (A/B switch, and always for a third order)
SECOND_ORDER = os.environ.get("TMDNET_TN_SECOND_ORDER", "hip")


def _double_backward(fwd, primals, gouts, ggs):
    """Second order of a first backward ``g -> VJP(fwd, primals, g)``: returns the gradients w.r.t.
    (gouts..., primals...) for the incoming ``ggs`` (one per primal), differentiating the composite
    ``fwd`` twice."""
    create = torch.is_grad_enabled()  # third order only when the caller builds a graph
    with torch.enable_grad():
        p = [None if x is None else x.detach().requires_grad_(True) for x in primals]
        g = [x.detach().requires_grad_(True) for x in gouts]
        live = [x for x in p if x is not None]
        outs = fwd(*p)
        outs = outs if isinstance(outs, (tuple, list)) else (outs,)
        first = torch.autograd.grad(outs, live, g, create_graph=True, allow_unused=True)
        it = iter(first)
        first_full = [None if x is None else next(it) for x in p]
        sel = [(f, gg) for f, gg in zip(first_full, ggs) if f is not None and gg is not None]
        if not sel:
            return [None] * (len(g) + len(p))
        second = torch.autograd.grad([f for f, _ in sel], g + live, [gg for _, gg in sel],
                                     create_graph=create, allow_unused=True)
    out = list(second[:len(g)])
    it = iter(second[len(g):])
    out += [None if x is None else next(it) for x in p]
    return out


# ----------------------------------------------------------------------------- Functions
class _NodeOp(Function):
    """One node pass.  ``fanout``: also returns an alias of the input ``a`` for a second consumer; that
    consumer's gradient arrives here and the backward kernel adds it (``gadd``), instead of the
    autograd engine summing the two gradients of ``a`` in a separate launch."""

    @staticmethod
    def forward(ctx, op, a, b, fanout):
        a = a.contiguous()
        b = None if b is None else b.contiguous()
        out = torch.empty(_out_shape(op, a), dtype=a.dtype, device=a.device)
        node_fwd_launch(op, a, b, out)
        ctx.op = op
        ctx.save_for_backward(a, b)
        if fanout:
            return out, a.view_as(a)
        return out

    @staticmethod
    def backward(ctx, gout, galias=None):
        a, b = ctx.saved_tensors
        if gout is None:
            gout = torch.zeros(_out_shape(ctx.op, a), dtype=a.dtype, device=a.device)
        gadd = None if galias is None else galias.contiguous()
        ga, gb = _NodeOpBwd.apply(ctx.op, gout.contiguous(), a, b, gadd)
        return None, ga, gb, None


class _NodeOpBwd(Function):
    @staticmethod
    def forward(ctx, op, gout, a, b, gadd):
        ga = torch.empty_like(a)
        gb = None if b is None else torch.empty_like(b)
        node_bwd_launch(op, a, b, gout, gadd, ga, gb)
        ctx.op = op
        ctx.has_add = gadd is not None
        ctx.save_for_backward(gout, a, b)
        return ga, gb

    @staticmethod
    def backward(ctx, gga, ggb):
        gout, a, b = ctx.saved_tensors
        op = ctx.op
        g_add = gga if ctx.has_add else None  # ga = VJP(gout) + gadd: identity in gadd
        if SECOND_ORDER != "composite" and not torch.is_grad_enabled() and a.is_cuda:
            # forward-over-reverse on dual numbers (tmdnet_tn_node_bwd2): d_gout = J (t_a, t_b),
            # (d_a, d_b) = H (t_a, t_b)
            need = ctx.needs_input_grad
            ta = None if gga is None else gga.contiguous()
            tb = None if (ggb is None or b is None) else ggb.contiguous()
            if ta is None and tb is None:
                return None, None, None, None, g_add
            d_g = torch.empty_like(gout) if need[1] else None
            d_a = torch.empty_like(a) if need[2] else None
            d_b = torch.empty_like(b) if (b is not None and need[3]) else None
            if d_g is not None or d_a is not None or d_b is not None:
                node_bwd2_launch(op, a, b, gout, ta, tb, d_g, d_a, d_b)
            return None, d_g, d_a, d_b, g_add
        if b is None:
            d = _double_backward(lambda x: op_composite(op, x), [a], [gout], [gga])
            return None, d[0], d[1], None, g_add
        d = _double_backward(lambda x, y: op_composite(op, x, y), [a, b], [gout], [gga, ggb])
        return None, d[0], d[1], d[2], g_add


def _apply(op, a, b=None, fanout=False):
    nat.require_gpu(a, "TensorNet node op")
    return _NodeOp.apply(op, a, b, fanout)


def pre(X, fanout=False):
    """Interaction input: X / (|X|^2 + 1), decomposed -> compact (tensornet.py:391-392).  ``fanout``:
    returns (compact, X alias) -- the alias for the residual, whose X-gradient the PRE backward adds."""
    return _apply(PRE, X, fanout=fanout)


def post(Yc, Mc, group):
    """Interaction update: decompose(msg Y + Y msg) (O(3)) or decompose(2 Y msg) (SO(3)), divided by
    |.|^2 + 1 (tensornet.py:398-406) -> compact."""
    return _apply(POST_O3 if group == "O(3)" else POST_SO3, Yc, Mc)


def resid(X, Dc):
    """X / (|X|^2 + 1) + dX + dX dX (tensornet.py:391, 410) -> full."""
    return _apply(RESID, X, Dc)


def norms(X):
    """cat(|I|^2, |A|^2, |S|^2) of decompose(X) (tensornet.py:230-231) -> [N, 3H]."""
    return _apply(NORMS, X)


def enorm(c, fanout=False):
    """tensor_norm(I + A + S) of a compact tensor (tensornet.py:317) -> [N, H] (``fanout``: and an alias
    of c for its second consumer, see pre)."""
    return _apply(ENORM, c, fanout=fanout)


def eout(c, f):
    """new_radial_tensor + I + A + S (tensornet.py:321-326): f [N, 3H] viewed as (N, H, 3) -> full."""
    return _apply(EOUT, c, f)


# ----------------------------------------------------------------------------- channel mixes
def _will_run(node):
    if node is None:
        return False
    try:
        return bool(torch._C._will_engine_execute_node(node))
    except RuntimeError:
        return True


def _blocks(t):
    """The I / A / S row blocks of a compact (9, N, H) tensor as 2-D GEMM operands."""
    N, H = t.shape[1], t.shape[2]
    return t[0], t[1:4].view(3 * N, H), t[4:9].view(5 * N, H)


def mix3_composite(c, w0, w1, w2):
    return torch.cat((torch.matmul(c[0:1], w0.t()), torch.matmul(c[1:4], w1.t()),
                      torch.matmul(c[4:9], w2.t())), dim=0)


class _Mix3(Function):
    """The reference's three per-part channel mixes (tensornet.py:318-320, 354-356, 372-374) on a
    compact tensor: three GEMMs writing the row blocks of one output buffer."""

    @staticmethod
    def forward(ctx, c, w0, w1, w2):
        c = c.contiguous()
        out = torch.empty((9, c.shape[1], w0.shape[0]), dtype=c.dtype, device=c.device)
        probs = [(src, w, True, None, dst, False) for src, w, dst in zip(_blocks(c), (w0, w1, w2), _blocks(out))]
        if c.is_cuda:  # one hand-written launch (x3 GEMMs above GEMM_MAX_ROWS rows; the library for fp64)
            kernels.gemm_group(probs)
        else:
            for src, w, _, _, dst, _ in probs:
                torch.mm(src, w.t(), out=dst)
        ctx.save_for_backward(c, w0, w1, w2)
        return out

    @staticmethod
    def backward(ctx, gout):
        c, w0, w1, w2 = ctx.saved_tensors
        nf = ctx.next_functions
        need_w = tuple(_will_run(nf[1 + i][0]) for i in range(3))
        return _Mix3Bwd.apply(need_w, gout.contiguous(), c, w0, w1, w2)


class _Mix3Bwd(Function):
    @staticmethod
    def forward(ctx, need_w, gout, c, w0, w1, w2):
        gc = torch.empty_like(c)
        ws = (w0, w1, w2)
        probs = [(g, w, False, None, dst, False) for g, w, dst in zip(_blocks(gout), ws, _blocks(gc))]
        if c.is_cuda:  # input gradients: one launch (x3 GEMMs above GEMM_MAX_ROWS rows)
            kernels.gemm_group(probs)
        else:
            for g, w, _, _, dst, _ in probs:
                torch.mm(g, w, out=dst)
        # weight gradients: one grouped TN launch (sums over the rows)
        gws = [torch.empty_like(w) if need else None for w, need in zip(ws, need_w)]
        tn = [{"A": g, "B": src, "C": gw} for g, src, gw in zip(_blocks(gout), _blocks(c), gws) if gw is not None]
        kernels.wgrad_tn(tn)
        ctx.save_for_backward(gout, c, w0, w1, w2)
        return (gc,) + tuple(gws)

    @staticmethod
    def backward(ctx, ggc, *ggw):
        gout, c, w0, w1, w2 = ctx.saved_tensors
        if SECOND_ORDER != "composite" and not torch.is_grad_enabled() and c.is_cuda:
            return (None,) + _mix3_second_order(ctx.needs_input_grad, gout, c, (w0, w1, w2), ggc, ggw)
        d = _double_backward(mix3_composite, [c, w0, w1, w2], [gout], [ggc] + list(ggw))
        return (None,) + tuple(d)


def _mix3_second_order(need, gout, c, ws, ggc, ggw):
    """VJP of (gc, gW_p) = (gout W_p, gout_p^T c_p) per row block p for cotangents (ggc, ggW_p) -- all GEMMs:
    d_gout_p = ggc_p W_p^T + c_p ggW_p^T,  d_c_p = gout_p ggW_p,  d_W_p = gout_p^T ggc_p."""
    ggw = [None if g is None else g.contiguous() for g in ggw]
    ggc = None if ggc is None else ggc.contiguous()
    gb, cb = _blocks(gout), _blocks(c)
    d_gout = d_c = None
    d_w = [None, None, None]
    if need[1] and (ggc is not None or any(g is not None for g in ggw)):
        d_gout = torch.empty_like(gout)
        probs = []
        for p, dst in enumerate(_blocks(d_gout)):
            first = True
            if ggc is not None:
                probs.append((_blocks(ggc)[p], ws[p], True, None, dst, False))
                first = False
            if ggw[p] is not None:
                probs.append((cb[p], ggw[p], True, None, dst, not first))
                first = False
            if first:
                dst.zero_()
        # the accumulating problems after the ones they add to (problems of one launch run in any order)
        kernels.gemm_group([q for q in probs if not q[5]])
        acc = [q for q in probs if q[5]]
        if acc:
            kernels.gemm_group(acc)
    if need[2] and any(g is not None for g in ggw):
        d_c = torch.zeros_like(c) if any(g is None for g in ggw) else torch.empty_like(c)
        kernels.gemm_group([(gb[p], ggw[p], False, None, dst, False)
                            for p, dst in enumerate(_blocks(d_c)) if ggw[p] is not None])
    if ggc is not None:
        tn = []
        for p in range(3):
            if need[3 + p]:
                d_w[p] = torch.empty_like(ws[p])
                tn.append({"A": gb[p], "B": _blocks(ggc)[p], "C": d_w[p]})
        kernels.wgrad_tn(tn)
    return (d_gout, d_c) + tuple(d_w)


def mix3(c, w0, w1, w2):
    return _Mix3.apply(c, w0, w1, w2)
