"""The ET interaction stack as ONE autograd node with a hand-scheduled backward.

Covers ``TorchMD_ET.forward``'s layer loop (reference models/torchmd_et.py:177-184) with every
``EquivariantMultiHeadAttention.forward`` inside it (torchmd_et.py:293-321).  Per layer the forward
is 7 launches:

    native_layer_norm -> [q|k|v] GEMM (one, on the stacked q/k/v weights) -> vec_proj GEMM
    -> [dk|dv] GEMM (one, on the stacked dk/dv weights) -> tmdnet_et_message_fwd -> o_proj GEMM
    -> tmdnet_et_epilogue_fwd (vec_dot, o-gating, both residuals)

and the backward, hand-scheduled on the same stream, 8-9 launches:

    tmdnet_et_epilogue_bwd -> g_o @ W_o -> tmdnet_et_message_bwd (gradients written straight into
    the stacked [q|k|v] / [dk|dv] gradient buffers; the vec residual and the cutoff / unit-vector
    gradients of all layers accumulated in-kernel) -> addmm_ into g_edge_attr (shared by all
    layers) -> addmm_ of the vec_proj backward into g_vec -> g_qkv @ W_qkv -> layer-norm backward.

Weight-gradient GEMMs run only when the current backward will actually deliver them (the
parameters' AccumulateGrad node is scheduled, ``torch._C._will_engine_execute_node``): a force
evaluation (``autograd.grad(E, pos, create_graph=True)``) skips them, ``loss.backward()`` computes
them.  The reference achieves none of this: it runs ~25 separate PyTorch kernels per layer forward
and autograd's generic per-op backward.

The backward is itself a Function so forces stay differentiable (training on forces); its own
backward (second order) recomputes the stack with composite PyTorch ops and differentiates twice.
"""
import contextlib
import os
import weakref

import torch
import torch.nn.functional as F
from torch.autograd import Function

from . import _native as nat
from . import kernels

_EPS = 1e-5  # nn.LayerNorm default (reference torchmd_et.py:223)


def _stack_views(params):
    """Make ``params`` (same trailing shape, same dtype/device) consecutive row blocks of one
    buffer, in place (``p.data`` becomes a view; Parameters, optimiser references and state_dict
    keys are unchanged).  Returns the buffer."""
    buf = torch.cat([p.detach() for p in params], 0)
    off = 0
    for p in params:
        n = p.shape[0]
        p.data = buf[off:off + n]
        off += n
    return buf


def _is_stacked(buf, params):
    if buf is None:
        return False
    es = buf.element_size()
    row = buf[0].numel() if buf.dim() > 1 else 1
    off = 0
    for p in params:
        if p.device != buf.device or p.dtype != buf.dtype or not p.is_contiguous() \
                or p.data_ptr() != buf.data_ptr() + off * row * es:
            return False
        off += p.shape[0]
    return off == buf.shape[0]


class LayerWeights:
    """Stacked views of one EquivariantMultiHeadAttention's projections.

    ``qkv_w`` [5H, H] = [q_proj; k_proj; v_proj] weights, ``dkv_w`` [(H|3H|4H), R] = [dk_proj;
    dv_proj]; the Parameters themselves alias row blocks of these buffers, so no per-step
    concatenation happens."""

    def __init__(self, layer):
        self.layer = layer
        self.bufs = {}

    def _get(self, name, params):
        buf = self.bufs.get(name)
        if not _is_stacked(buf, params):
            buf = _stack_views(params)
            self.bufs[name] = buf
        return buf

    def fused(self):
        L = self.layer
        qkv_w = self._get("qkv_w", [L.q_proj.weight, L.k_proj.weight, L.v_proj.weight])
        qkv_b = self._get("qkv_b", [L.q_proj.bias, L.k_proj.bias, L.v_proj.bias])
        return qkv_w, qkv_b


class StackWeights:
    """The dk/dv projections of ALL layers as row blocks of one [L*D, R] weight (D = H | 3H | 4H)
    and one [L*D] bias: layer l's [dk; dv] is rows [l*D, (l+1)*D).  They only read the edge
    features, so small systems compute every layer's projection with ONE GEMM up front (and the
    edge-feature gradient with one GEMM at the end of the backward)."""

    def __init__(self, layers):
        self.layers = layers
        self.bufs = {}

    def _get(self, name, params):
        buf = self.bufs.get(name)
        if not _is_stacked(buf, params):
            buf = _stack_views(params)
            self.bufs[name] = buf
        return buf

    def dkv(self):
        mods = [m for layer in self.layers for m in (layer.dk_proj, layer.dv_proj) if m is not None]
        if not mods:
            return None, None
        return self._get("w", [m.weight for m in mods]), self._get("b", [m.bias for m in mods])


# Batch every layer's dk/dv projection into one GEMM while its output (E x L*D fp32) stays below this.
BATCH_DKV_BYTES = 2 << 30
# From this many edges on, v / dv rows are produced in the planar layout [x | v1 | v2] (H-blocks,
# TMDNET_ET_V_PLANAR) by permuting the weight rows once per forward: contiguous row segments for the
# edge kernels' 16-byte loads (+4-7 % on the C5 forward); below it the two small gathers are not worth it.
PLANAR_MIN_EDGES = 131072
# dk/dv projection rows shared by the two directions of an edge pair (halves the projection GEMM)
PAIR_ROWS = True
# dk/dv projection FUSED into the edge kernels (et_fused.hip: tmdnet_et_fused_fwd_f32 / _bwd_f32) for a
# fixed RBF basis of r (H = 128, 8 heads, SiLU, both projections): the projection rows are never written
# (C5: 2.8 GB per layer, read back once per direction by the unfused kernels; the force pass's
# d(dk,dv)/dr rows likewise).  TMDNET_FEP=0 turns it off.
FEP = os.environ.get("TMDNET_FEP", "auto")
# ... on graphs from this many edges (below it -- the QM9 batches -- the per-layer kernels are latency-bound:
# C2 measured 1.39 ms fused vs 0.90 ms unfused per energy + force step, r04)
FEP_MIN_EDGES = int(os.environ.get("TMDNET_FEP_MIN_EDGES", "131072"))
# When a backward can follow (grad enabled), how it gets the projection: "fused" (default) = the
# force-pass (dr mode) backward is fused the same way (d pre / d r formed on the MFMA in-kernel); a
# backward that needs the projection rows (parameter gradients, the recorded force pass of force-matching
# training) forms them by the GEMM then ("lazy" for every backward); "off" = with a backward to follow,
# the forward is the unfused one (projection GEMM + message kernel).  Force-matching training steps
# (second_order_expected) always run the unfused forward: their backward reads the rows.
FEP_BWD = os.environ.get("TMDNET_FEP_BWD", "fused")
FUSED_BWD = FEP_BWD == "fused"
# "dr mode" force pass (see _backward_layers): on whenever the force pass needs no weight gradient
# and the features are a fixed basis of r (also under create_graph, which the reference force pass
# always uses: the second order then re-forms f from r by the composite basis).  Measured on
# MI355X: C2 1.076 -> 1.063 ms, C4 0.932 -> 0.917 ms, C5 73.9 -> 71.3 ms; the eager training step
# is within its run-to-run noise (29-35 ms).  TMDNET_DR=0 turns it off.
DR_MODE = os.environ.get("TMDNET_DR", "auto")
# second order of the force pass (force-matching training): "hand" = the hand-scheduled adjoint
# (_second_order), "composite" = autograd over the recomputed stack (the reference for tests / A-B)
SECOND_ORDER = os.environ.get("TMDNET_ET_SECOND_ORDER", "hand")
# under create_graph the force pass itself runs in the recorded training form (g_r = <g_f, df/dr>) and
# hands its record to the hand second order, which then skips re-running it.  TMDNET_ET_RECORD=0: the
# dr-mode force pass + a recorded re-run inside the second order (the previous scheme, for A/B)
RECORD_IN_FORCE_PASS = os.environ.get("TMDNET_ET_RECORD", "1") not in ("0", "off")
# ... but only inside ``second_order_expected()`` (the training steps): the reference force pass always
# builds its graph (create_graph=True), so create_graph alone does not say a second backward follows,
# and an energy+force evaluation must keep the cheaper dr-mode force pass
_EXPECT_SECOND_ORDER = [False]
# the projection's weight gradient over the edge rows (K = E, a 4096 x 64 output: FLOP-bound on the
# fp32 MFMA): "tn" = one split-K launch of the 16-byte-load TN kernel, bias included (ET-QM9 step:
# 215 us; the scalar TN kernel took 500), "lib" = library GEMMs + a column sum (243 + 54 us)
PROJ_WGRAD = os.environ.get("TMDNET_PROJ_WGRAD", "tn")
# the node weights' gradients (per layer [q|k|v], o_proj, vec_proj, LayerNorm, over the atoms): "tn" =
# grouped split-K TN GEMMs with the bias columns, "bmm" = batched library GEMMs + reductions
NODE_WGRAD = os.environ.get("TMDNET_NODE_WGRAD", "tn")


@contextlib.contextmanager
def second_order_expected(on=True):
    """Declare that the force pass(es) run inside will be differentiated again (force-matching
    training): the ET stack's force pass then records what the hand second order needs."""
    prev = _EXPECT_SECOND_ORDER[0]
    _EXPECT_SECOND_ORDER[0] = bool(on)
    try:
        yield
    finally:
        _EXPECT_SECOND_ORDER[0] = prev

_PERMS = {}


def _v_perm(H, heads, device):
    """Row j of the planar [x | v1 | v2] block = row perm[j] of the reference per-head interleave
    [h][x|v1|v2] (torchmd_et.py:282-291, 299-303)."""
    key = ("v", H, heads, str(device))
    if key not in _PERMS:
        d = H // heads
        j = torch.arange(3 * H)
        part, rem = j // H, j % H
        _PERMS[key] = (rem // d * 3 * d + part * d + rem % d).to(device)
    return _PERMS[key]


def _planar_perms(meta, device):
    """(qkv row perm, its inverse, all-layer dk/dv row perm, its inverse) for the planar layout."""
    key = ("stack", meta.H, meta.heads, meta.n_layers, meta.hk, meta.hv, str(device))
    if key not in _PERMS:
        H = meta.H
        vp = _v_perm(H, meta.heads, device)
        qkv = torch.cat([torch.arange(2 * H, device=device), 2 * H + vp])
        per = ([torch.arange(H, device=device)] if meta.hk else []) + \
            ([H * int(meta.hk) + vp] if meta.hv else [])
        one = torch.cat(per) if per else torch.zeros(0, dtype=torch.long, device=device)
        dkv = torch.cat([l * meta.D + one for l in range(meta.n_layers)])
        inv = lambda p: torch.empty_like(p).scatter_(0, p, torch.arange(p.numel(), device=device))  # noqa
        _PERMS[key] = (qkv, inv(qkv), dkv, inv(dkv), one, inv(one))
    return _PERMS[key]


def layer_params(layer):
    """Flat parameter list of one layer, in the order the stack Function consumes it."""
    ps = [layer.layernorm.weight, layer.layernorm.bias, layer.q_proj.weight, layer.q_proj.bias,
          layer.k_proj.weight, layer.k_proj.bias, layer.v_proj.weight, layer.v_proj.bias,
          layer.vec_proj.weight, layer.o_proj.weight, layer.o_proj.bias]
    if layer.dk_proj is not None:
        ps += [layer.dk_proj.weight, layer.dk_proj.bias]
    if layer.dv_proj is not None:
        ps += [layer.dv_proj.weight, layer.dv_proj.bias]
    return ps


class _Meta:
    """Non-tensor context of one stack call."""

    def __init__(self, graph, heads, H, hk, hv, n_layers, fused, acc_nodes=None, dkv_w=None, dkv_b=None,
                 batched=False):
        self.graph = graph
        self.heads = heads
        self.H = H
        self.hk = hk
        self.hv = hv
        self.n_layers = n_layers
        self.fused = fused  # per layer (qkv_w, qkv_b) stacked views
        self.D = (int(hk) + 3 * int(hv)) * H  # dk/dv rows per layer
        self.dkv_w, self.dkv_b = dkv_w, dkv_b  # all layers' [dk; dv] (StackWeights)
        self.batched = batched  # one GEMM for every layer's projection
        self.planar = False     # TMDNET_ET_V_PLANAR row layout for v / dv (set by et_stack)
        self.flags = 0
        self.acts = 0           # kernels.et_act_flags of the layers' activations (0: SiLU / SiLU)
        self.qkv_eff = fused    # the weights the GEMMs use (row-permuted copies when planar)
        self.dkv_eff = (dkv_w, dkv_b)
        self.np = 11 + 2 * int(hk) + 2 * int(hv)  # parameters per layer
        self.pairs = None       # (pair_row, pair_edge) of the graph: pair-shared dk/dv rows
        self.pk_rows = None
        self.rbf = None         # (mu, beta, cutoff_lower, cutoff_upper, rbf_type): f = rbf(r) ("dr mode")
        self.out_norm = False   # the model's final LayerNorm fused into the last epilogue (2 trailing params)
        self.f_pairs = None     # f at the pair rows, when the caller produced it with the features
        self.fdp_pairs = None   # ... and d f / d r there (the dr-mode force pass's operand)
        self.dkv_wp = None      # the bf16 split of dkv_eff[0] (dkv_split), once per forward
        self.fep = False        # the forward runs the fused-projection edge kernel (FEP)
        self.fep_imgs = None    # per layer: its weight image (kernels.fep_split), made by the forward
        self.grad_mode = True   # torch.is_grad_enabled() where the stack was called (a backward can follow)

    def split(self, params):
        return [params[i * self.np:(i + 1) * self.np] for i in range(self.n_layers)]

    def dkv_split(self):
        """The exact bf16 split of the stacked dk/dv weight (kernels.proj_split), made once per forward
        and shared by the projection, its r-derivative and the second-order adjoint."""
        if self.dkv_wp is None and self.dkv_eff[0] is not None:
            self.dkv_wp = kernels.proj_split(self.dkv_eff[0])
        return self.dkv_wp

    def dkv_proj(self, A, l=None, bias=True):
        """A @ W.T (+ b) for the stacked dk/dv weight (l None) or layer l's rows of it."""
        w, b = self.dkv_eff if l is None else self.dkv_layer(l)
        return kernels.proj(A, w, b if bias else None, wp=self.dkv_split(), row0=0 if l is None else l * self.D)

    def dkv_layer(self, l):
        w, b_ = self.dkv_eff
        if w is None:
            return None, None
        a, b = l * self.D, (l + 1) * self.D
        return w[a:b], b_[a:b]

    def refresh_effective(self):
        """Row-permuted copies of the stacked weights for the planar layout (once per forward, so
        in-place parameter updates are always seen; two small gathers per layer)."""
        self.dkv_wp = None
        if not self.planar:
            self.qkv_eff, self.dkv_eff = self.fused, (self.dkv_w, self.dkv_b)
            return
        qp, _, dp, _, _, _ = self.perms
        self.qkv_eff = [(w.index_select(0, qp), b.index_select(0, qp)) for w, b in self.fused]
        self.dkv_eff = (self.dkv_w.index_select(0, dp), self.dkv_b.index_select(0, dp)) \
            if self.dkv_w is not None else (None, None)


def _epilogue_fwd(x, vec, vecp, o, veca):
    lib = nat.load()
    N, H = x.shape
    xo = torch.empty_like(x)
    vo = torch.empty_like(veca)
    rc = lib.tmdnet_et_epilogue_fwd(nat.dtype_code(x.dtype), N, H, nat.ptr(x), nat.ptr(vec),
                                    nat.ptr(vecp), nat.ptr(o), nat.ptr(veca), nat.ptr(xo), nat.ptr(vo),
                                    nat.stream(x.device))
    nat.check(rc, "tmdnet_et_epilogue_fwd")
    return xo, vo


def _epilogue_bwd(gx, gvec, vecp, o, g_vecp, g_o, acc=False):
    """tmdnet_et_epilogue_bwd_acc: g_vecp / g_o written (acc: added to -- they hold injected cotangents)."""
    lib = nat.load()
    N, H = gx.shape
    rc = lib.tmdnet_et_epilogue_bwd_acc(nat.dtype_code(gx.dtype), N, H, nat.ptr(gx), nat.ptr(gvec),
                                        nat.ptr(vecp), nat.ptr(o), nat.ptr(g_vecp), nat.ptr(g_o), int(acc),
                                        nat.stream(gx.device))
    nat.check(rc, "tmdnet_et_epilogue_bwd_acc")


def _epi_ln(x, vec, vecp, o, veca, ln_w, ln_b, xn_out=None, vo_out=None):
    """tmdnet_et_epilogue_ln_fwd: this layer's epilogue (o not None) and the next layer's LayerNorm
    in one pass.  Returns (x_out, vec_out, xn, mean, rstd); o None: LayerNorm of x only.  xn_out /
    vo_out: caller buffers for xn / vec_out (the layer-stacked activations)."""
    lib = nat.load()
    N, H = x.shape
    xo = torch.empty_like(x) if o is not None else None
    vo = (vo_out if vo_out is not None else torch.empty_like(veca)) if o is not None else None
    xn = xn_out if xn_out is not None else torch.empty_like(x)
    mean = torch.empty((N, 1), dtype=x.dtype, device=x.device)
    rstd = torch.empty((N, 1), dtype=x.dtype, device=x.device)
    rc = lib.tmdnet_et_epilogue_ln_fwd(nat.dtype_code(x.dtype), N, H, nat.ptr(x), nat.ptr(vec), nat.ptr(vecp),
                                       nat.ptr(o), nat.ptr(veca), nat.ptr(ln_w), nat.ptr(ln_b), _EPS,
                                       nat.ptr(xo), nat.ptr(vo), nat.ptr(xn), nat.ptr(mean), nat.ptr(rstd),
                                       nat.stream(x.device))
    nat.check(rc, "tmdnet_et_epilogue_ln_fwd")
    return xo, vo, xn, mean, rstd


# The forward's node mixes with the epilogue / LayerNorm pass folded in (et_nodemix.hip): per layer
# tmdnet_et_ln_mix_f32 (LayerNorm + [q|k|v] + vec_proj) and tmdnet_et_oproj_epilogue_f32 (o_proj + the
# epilogue) instead of [q|k|v]/vec_proj GEMM + o_proj GEMM + epilogue-LayerNorm pass: one launch per layer
# fewer.  fp32, H % 64 == 0, H <= 256, in the small grouped GEMM's regime (3N rows <= GEMM_MAX_ROWS; larger
# systems keep the x3 GEMMs).  TMDNET_ET_NODE_FUSE=0 keeps the three-launch form.
NODE_FUSE = os.environ.get("TMDNET_ET_NODE_FUSE", "1") != "0"


def _node_fuse_ok(x):
    N, H = x.shape
    return (NODE_FUSE and x.is_cuda and x.dtype == torch.float32 and H % 64 == 0 and H <= 256
            and 3 * N <= kernels.GEMM_MAX_ROWS)


def _ln_mix(x, ln_w, ln_b, w, b, vec, vec_w, xn_out):
    """tmdnet_et_ln_mix_f32: (qkv, vecp, xn, mean, rstd) with xn written into ``xn_out``."""
    lib = nat.load()
    N, H = x.shape
    qkv = torch.empty((N, w.shape[0]), dtype=x.dtype, device=x.device)
    mean = torch.empty((N, 1), dtype=x.dtype, device=x.device)
    rstd = torch.empty((N, 1), dtype=x.dtype, device=x.device)
    vecp = torch.empty((N, 3, vec_w.shape[0]), dtype=x.dtype, device=x.device) if vec is not None else None
    w, ln_w, ln_b = w.contiguous(), ln_w.contiguous(), ln_b.contiguous()
    vec_w = vec_w.contiguous() if vec is not None else None
    rc = lib.tmdnet_et_ln_mix_f32(N, H, nat.ptr(x), nat.ptr(ln_w), nat.ptr(ln_b), _EPS, nat.ptr(w), nat.ptr(b),
                                  w.shape[0], nat.ptr(qkv), nat.ptr(xn_out), nat.ptr(mean), nat.ptr(rstd),
                                  nat.ptr(vec), nat.ptr(vec_w), vec_w.shape[0] if vec is not None else 0,
                                  nat.ptr(vecp), nat.stream(x.device))
    nat.check(rc, "tmdnet_et_ln_mix_f32")
    return qkv, vecp, xn_out, mean, rstd


def _oproj_epi(xa, o_w, o_b, x, vec, vecp, veca, vo_out):
    """tmdnet_et_oproj_epilogue_f32: (o, x_out, vec_out) with vec_out written into ``vo_out``."""
    lib = nat.load()
    N, H = x.shape
    o = torch.empty((N, o_w.shape[0]), dtype=x.dtype, device=x.device)
    xo = torch.empty_like(x)
    o_w = o_w.contiguous()
    rc = lib.tmdnet_et_oproj_epilogue_f32(N, H, nat.ptr(xa), nat.ptr(o_w), nat.ptr(o_b), nat.ptr(x), nat.ptr(vec),
                                          nat.ptr(vecp), nat.ptr(veca), nat.ptr(o), nat.ptr(xo), nat.ptr(vo_out),
                                          nat.stream(x.device))
    nat.check(rc, "tmdnet_et_oproj_epilogue_f32")
    return o, xo, vo_out


def _ln_bwd_oproj(g_xn, x, mean, rstd, ln_w, g_res, g_vec, vecp, o, o_w, g_vecp, g_o):
    """tmdnet_et_lnbwd_oproj_f32: (g_x, g_xa) -- the LayerNorm backward of a layer (+ residual g_res), the
    previous layer's epilogue backward into g_vecp / g_o, and that layer's g_xa = g_o W_o (H = 128)."""
    lib = nat.load()
    N, H = x.shape
    gx = torch.empty_like(x)
    gxa = torch.empty_like(x)
    rc = lib.tmdnet_et_lnbwd_oproj_f32(N, H, nat.ptr(g_xn), nat.ptr(x), nat.ptr(mean), nat.ptr(rstd), nat.ptr(ln_w),
                                       nat.ptr(g_res), nat.ptr(g_vec), nat.ptr(vecp), nat.ptr(o), nat.ptr(o_w),
                                       nat.ptr(gx), nat.ptr(g_vecp), nat.ptr(g_o), nat.ptr(gxa), nat.stream(x.device))
    nat.check(rc, "tmdnet_et_lnbwd_oproj_f32")
    return gx, gxa


def _ln_bwd_epi(g_xn, x, mean, rstd, ln_w, g_res, g_vec, vecp, o, g_vecp, g_o, wrows=None, g_res2=None, acc=False):
    """tmdnet_ln_bwd_epilogue_w: g_x = g_res + LayerNorm backward (g_res None: no residual), then the
    previous layer's epilogue backward into g_vecp / g_o (o None: skipped); ``wrows`` (optional
    [N, H]) receives g_xn * xhat, the row terms of the LayerNorm weight gradient; g_res2: a second
    residual term; acc: g_vecp / g_o are added to (they hold injected cotangents)."""
    lib = nat.load()
    N, H = x.shape
    g_x = torch.empty_like(g_xn)
    rc = lib.tmdnet_ln_bwd_epilogue_w(nat.dtype_code(x.dtype), N, H, nat.ptr(g_xn), nat.ptr(x), nat.ptr(mean),
                                      nat.ptr(rstd), nat.ptr(ln_w), nat.ptr(g_res), nat.ptr(g_res2), nat.ptr(g_x),
                                      nat.ptr(g_vec), nat.ptr(vecp), nat.ptr(o), nat.ptr(g_vecp), nat.ptr(g_o),
                                      nat.ptr(wrows), int(acc), nat.stream(x.device))
    nat.check(rc, "tmdnet_ln_bwd_epilogue_w")
    return g_x


def _pair_f(meta, f):
    """The edge features at the projection rows (the pair rows when the graph has them)."""
    if meta.pairs is None:
        return f
    return meta.f_pairs if meta.f_pairs is not None else f.index_select(0, meta.pairs[1])


def _act_pkv(meta, acts, l, f):
    """Layer l's forward activations, with its projection rows formed now if the fused forward (FEP)
    skipped them (a backward that contracts them: training form, or the unfused dr-mode pass)."""
    a = acts[l]
    if a[7] is None and meta.fep_imgs is not None and meta.D:
        if meta.batched:  # every layer's rows in one GEMM, as the unfused forward lays them out: the
            # message backward reads d(dk,dv)/dr with the projection rows' leading dimension
            pkv_all, D = meta.dkv_proj(_pair_f(meta, f)), meta.D
            for j in range(meta.n_layers):
                acts[j] = acts[j][:7] + (pkv_all[:, j * D:(j + 1) * D],) + acts[j][8:]
        else:
            acts[l] = a[:7] + (meta.dkv_proj(_pair_f(meta, f), l),) + a[8:]
    return acts[l]


def _forward_layers(meta, x, f, C, u, params, r=None, want_bwd=False):
    """HIP/GEMM forward; returns outputs and the per-layer activations the backward needs."""
    H = meta.H
    N = x.shape[0]
    vec = None
    acts = []
    D = meta.D
    meta.refresh_effective()
    # the projections depend on |r| only: one row per edge PAIR ((E + N) / 2 rows), read by both
    # directions through pk_rows (bit-identical to the per-edge projection)
    fep = meta.fep and r is not None and (not want_bwd or (FEP_BWD != "off" and not _EXPECT_SECOND_ORDER[0]))
    if not fep:
        meta.fep_imgs = None  # (the backward's fused path keys on them: none from an earlier forward)
    fp = _pair_f(meta, f) if (D and not fep) else f
    pkv_all = meta.dkv_proj(fp) if (meta.batched and D and not fep) else None
    layers = meta.split(params)
    L = len(layers)
    od = dict(dtype=x.dtype, device=x.device)
    # the activations the weight gradients multiply, stacked over layers (one batched GEMM per weight
    # kind in the backward): layer l's LayerNorm output, aggregated x and vec input (layer 0: none)
    xn_all, xa_all = torch.empty((L, N, H), **od), torch.empty((L, N, H), **od)
    vec_all = torch.empty((L, N, 3, H), **od)
    meta.stk = (xn_all, xa_all, vec_all)
    # layer l's LayerNorm is computed by layer l-1's epilogue kernel (layer 0: LayerNorm alone) -- or, in the
    # node-fused form, by layer l's [q|k|v] mix (tmdnet_et_ln_mix_f32)
    nf = _node_fuse_ok(x)
    if not nf:
        _, _, xn, mean, rstd = _epi_ln(x, None, None, None, None, layers[0][0], layers[0][1], xn_out=xn_all[0])
    for l, p in enumerate(layers):
        vec_w, o_w, o_b = p[8], p[9], p[10]
        qkv_w, qkv_b = meta.qkv_eff[l]
        dkv_w, dkv_b = meta.dkv_layer(l)
        if nf:  # LayerNorm + [q|k|v] + vec_proj, one launch
            qkv, vecp, xn, mean, rstd = _ln_mix(x, p[0], p[1], qkv_w, qkv_b, vec, vec_w, xn_all[l])
        else:
            # [q|k|v] and vec_proj in ONE launch (tmdnet_gemm_f32; library GEMMs outside its envelope)
            qkv = torch.empty((N, qkv_w.shape[0]), dtype=x.dtype, device=x.device)
            probs = [(xn, qkv_w, True, qkv_b, qkv, False)]
            vecp = None
            if vec is not None:
                vecp = torch.empty((N, 3, 3 * H), dtype=x.dtype, device=x.device)
                probs.append((vec.view(3 * N, H), vec_w, True, None, vecp.view(3 * N, 3 * H), False))
            kernels.gemm_group(probs)
        xa = xa_all[l]
        veca = torch.empty((N, 3, H), dtype=x.dtype, device=x.device)
        if fep:  # projection fused into the edge kernel (no rows: a backward that needs them forms them)
            pkv = None
            if l == 0:
                meta.fep_imgs = []
                # the RBF fragments of the evaluation (pair rows), shared by every layer's fused kernels
                # (the fused neighbour embedding's, when it made them already: kernels.fep_frag_shared)
                meta.fep_frag = kernels.fep_frag_shared(meta.graph, r, meta.rbf)
            if not meta.planar:  # the image's rows are always in the planar [dk | dv_x | dv_1 | dv_2] order
                one = _planar_perms(meta, x.device)[4]
                dkv_w, dkv_b = dkv_w.index_select(0, one), dkv_b.index_select(0, one)
            meta.fep_imgs.append(kernels.fep_split(dkv_w, dkv_b))
            kernels.et_fused_fwd_launch(qkv[:, :H], qkv[:, H:2 * H], qkv[:, 2 * H:], vec, C, u,
                                        meta.fep_imgs[l], meta.fep_frag, meta.graph, meta.heads, xa, veca,
                                        flags=meta.flags)
        else:
            if pkv_all is not None:
                pkv = pkv_all[:, l * D:(l + 1) * D]
            else:
                pkv = meta.dkv_proj(fp, l) if dkv_w is not None else None
            pk = pkv[:, :H] if meta.hk else None
            pv = pkv[:, H * int(meta.hk):] if meta.hv else None
            kernels.et_message_fwd_launch(qkv[:, :H], qkv[:, H:2 * H], qkv[:, 2 * H:], vec, pk, pv, C, u,
                                          meta.graph, meta.heads, xa, veca, meta.flags, meta.pk_rows)
        if nf and l + 1 < len(layers):  # o_proj + the epilogue, one launch (the next LayerNorm: its mix)
            o, x_next, vec_next = _oproj_epi(xa, o_w, o_b, x, vec, vecp, veca, vec_all[l + 1])
            acts.append((x, vec, xn, mean, rstd, qkv, vecp, pkv, xa, o))
            x, vec = x_next, vec_next
            continue
        o = torch.empty((N, o_w.shape[0]), dtype=x.dtype, device=x.device)
        kernels.gemm_group([(xa, o_w, True, o_b, o, False)])
        acts.append((x, vec, xn, mean, rstd, qkv, vecp, pkv, xa, o))
        if l + 1 < len(layers):
            x, vec, xn, mean, rstd = _epi_ln(x, vec, vecp, o, veca, layers[l + 1][0], layers[l + 1][1],
                                             xn_out=xn_all[l + 1], vo_out=vec_all[l + 1])
        elif meta.out_norm:  # last epilogue + the model's out_norm (torchmd_et.py:186) in one kernel
            x_pre, vec, x, mean, rstd = _epi_ln(x, vec, vecp, o, veca, params[-2], params[-1])
            acts.append((x_pre, mean, rstd))
        else:
            x, vec = _epilogue_fwd(x, vec, vecp, o, veca)
    return x, vec, acts


def _backward_layers(meta, gX, gV, f, C, u, params, acts, need_ws, r=None, dr=False, record=None, inject=None,
                     seed_pre_norm=False, want_f=True):
    """Hand-scheduled first-order backward.  Returns (g_x, g_f, g_C, g_u, g_r, g_params).

    ``dr`` ("dr mode", the force pass: no weight gradients, f = rbf(r)): the projection gradient is
    never materialised.  d pkv / d r = (d f / d r) W^T is formed once per pair row (one GEMM the
    size of the forward projection) and the message backward contracts the per-edge projection
    gradient with it in-kernel, accumulating g_r -- instead of writing the E x (layers * D) gradient
    and reading it back through the edge-feature GEMM.  g_f is then None.

    For the hand-scheduled second order (``_second_order``):
      * ``record`` (a list): every layer's backward intermediates are kept in fresh buffers and
        appended as a dict (layer L-1 first): the seeds gX / gV the layer's step receives, g_o,
        g_vecp, g_xa, g_qkv, g_xn; and ``record`` gets the attribute-like entry {"g_pkv": ...} last;
      * ``inject`` (dict of per-layer lists): extra cotangents of the forward's intermediates added
        where the backward forms their gradients -- "o", "vecp", "qkv" (node), "pkv" (edge rows of
        the layer's projection), "vec" (the layer's vec input), "x" (the layer's x input);
      * ``seed_pre_norm``: with the fused out_norm, gX is the gradient of the norm's INPUT (skip its
        backward);
      * ``want_f`` False: the edge-feature gradient g_f is not formed (a training step's parameter
        backward never consumes it: f = rbf(r) has no parameters) -- one E x (layers * D) GEMM fewer."""
    H = meta.H
    N = gX.shape[0]
    graph = meta.graph
    E = graph.n_edges
    o = dict(dtype=gX.dtype, device=gX.device)
    has_e = meta.hk or meta.hv
    D = meta.D
    rec = record is not None
    inj = inject or {}
    stk = inj.get("stk")  # the second order's layer-stacked injections (see below)
    acc = stk is not None

    def injected(key, l):
        lst = inj.get(key)
        return None if lst is None else lst[l]

    # the kernels accumulate the edge gradients (g_C, g_u, g_r) across layers into one buffer; the
    # first layer of the backward overwrites it (every slot, padding included): no zero fill
    zbuf = torch.empty(((5 if dr else 4) * E,), **o)
    g_C, g_u = zbuf[:E], zbuf[E:4 * E].view(E, 3)
    g_r = None
    # the fused force-pass backward (tmdnet_et_fused_bwd_f32) after a fused forward: d pre / d r formed
    # in-kernel, no projection rows at all
    fused = (dr and meta.fep and not rec and not inj and meta.fep_imgs is not None and FUSED_BWD
             and all(a[7] is None for a in acts[:meta.n_layers]))
    if dr:
        assert has_e and not any(need_ws) and meta.rbf is not None
        g_r = zbuf[4 * E:]
        if not fused:
            if meta.fdp_pairs is not None and meta.pairs is not None:
                fdp = meta.fdp_pairs
            else:
                fdp = kernels.rbf_deriv(r, *meta.rbf, rows=meta.pairs[1] if meta.pairs is not None else None)
            dpkv_all = meta.dkv_proj(fdp, bias=False) if meta.batched else None
    # dr mode recorded (the create_graph force pass): g_r in-kernel AND the projection gradient kept
    # padding rows of a static-capacity list are zeroed by the kernel: no memset needed
    if has_e and (not dr or rec):
        if acc and stk.get("pkv") is not None and (meta.batched or rec):
            g_pkv_all = stk["pkv"]  # [E, layers * D], accumulated into
        else:
            g_pkv_all = torch.empty((E, meta.n_layers * D if (meta.batched or rec) else D), **o)
    g_f = None
    new = lambda shape: torch.empty(shape, **o)  # noqa: E731
    L = meta.n_layers
    # per-layer gradients stacked over layers: the record keeps every layer's, and the weight
    # gradients are formed for all layers at once after the loop (_node_weight_grads)
    # the second order's injected cotangents of the forward intermediates (o, vecp, [q|k|v], the
    # projection rows) arrive as layer-stacked buffers: the gradients are ACCUMULATED into them by the
    # kernels (no separate adds)
    if acc:
        g_qkv_all, g_o_all, g_vecp_all = stk["qkv"], stk["o"], stk["vecp"]
    else:
        g_qkv_all, g_o_all, g_vecp_all = new((L, N, 5 * H)), new((L, N, 3 * H)), new((L, N, 3, 3 * H))
    g_xn_all = new((L, N, H))
    any_w = any(need_ws[:L])
    ln_rows = new((L, N, H)) if any_w else None
    gvec_bufs = [new((N, 3, H)), new((N, 3, H))]
    layers = meta.split(params)
    g_params = [None] * len(params)
    epi_done = False  # this layer's epilogue backward already ran (fused into the next layer's LN bwd)
    # the node-fused backward (tmdnet_et_lnbwd_oproj_f32): each LayerNorm backward also runs the layer
    # below's epilogue backward and its o_proj input gradient g_xa (no injections, no weight rows)
    bwd_nf = (not acc and not inj and not any(need_ws[:meta.n_layers + 1]) and gX is not None and H == 128
              and _node_fuse_ok(gX))
    g_xa_pre = None  # the next (lower) layer's g_xa, formed by the fused kernel
    x_top = inj.get("x_top")  # a cotangent of the last epilogue's output (the out_norm input)
    if meta.out_norm and not seed_pre_norm:  # gX is the gradient of LN(x_out): back through out_norm first
        x_pre, mean_o, rstd_o = acts[meta.n_layers]
        last = acts[meta.n_layers - 1]
        if need_ws[meta.n_layers]:  # LayerNorm backward (+ the injected cotangent) and its weight gradients
            g_y = gX
            gX = _ln_bwd_epi(g_y, x_pre, mean_o, rstd_o, params[-2], x_top, None, None, None, None, None)
            g_params[-2:] = list(kernels.layer_norm_wgrad(g_y, x_pre, mean_o, rstd_o))
        elif x_top is not None:  # LayerNorm backward + the injected cotangent (epilogue in the loop)
            gX = _ln_bwd_epi(gX, x_pre, mean_o, rstd_o, params[-2], x_top, None, None, None, None, None)
        elif bwd_nf and gV is not None:  # ... and the last layer's o_proj input gradient, one kernel
            gX, g_xa_pre = _ln_bwd_oproj(gX, x_pre, mean_o, rstd_o, params[-2], None, gV, last[6], last[9],
                                         layers[L - 1][9], g_vecp_all[L - 1], g_o_all[L - 1])
            epi_done = True
        else:  # LayerNorm backward + the last layer's epilogue backward, one kernel
            gX = _ln_bwd_epi(gX, x_pre, mean_o, rstd_o, params[-2], None, gV, last[6], last[9], g_vecp_all[L - 1],
                             g_o_all[L - 1])
            epi_done = True
    elif x_top is not None:
        gX = gX + x_top
    for l in reversed(range(meta.n_layers)):
        p = layers[l]
        x, vec, xn, mean, rstd, qkv, vecp, pkv, xa, o_ = acts[l] if fused else _act_pkv(meta, acts, l, f)
        ln_w, ln_b = p[0], p[1]
        vec_w, o_w = p[8], p[9]
        qkv_w, _ = meta.qkv_eff[l]
        dkv_w, _ = meta.dkv_layer(l)
        g_qkv, g_o, g_vecp = g_qkv_all[l], g_o_all[l], g_vecp_all[l]
        gpk = gpv = dpk = dpv = None
        if dr and not fused:
            dpkv = dpkv_all[:, l * D:(l + 1) * D] if meta.batched else meta.dkv_proj(fdp, l, bias=False)
            dpk = dpkv[:, :H] if meta.hk else None
            dpv = dpkv[:, H * int(meta.hk):] if meta.hv else None
        if has_e and (not dr or rec):
            g_pkv = g_pkv_all[:, l * D:(l + 1) * D] if (meta.batched or rec) else g_pkv_all
            if acc and not (meta.batched or rec):  # per-layer buffer (row stride D): start from the injection
                g_pkv.copy_(stk["pkv"][:, l * D:(l + 1) * D])
            gpk = g_pkv[:, :H] if meta.hk else None
            gpv = g_pkv[:, H * int(meta.hk):] if meta.hv else None
        if rec:
            step = {"gX": gX, "gV": gV}
        if not epi_done:
            _epilogue_bwd(gX, gV, vecp, o_, g_vecp, g_o, acc=acc)
        if not acc and injected("o", l) is not None:
            g_o.add_(injected("o", l))
            if vecp is not None:
                g_vecp.add_(injected("vecp", l))
        if g_xa_pre is not None:
            g_xa, g_xa_pre = g_xa_pre, None
        else:
            g_xa = torch.empty((N, H), **o)
            kernels.gemm_group([(g_o, o_w, False, None, g_xa, False)])
        g_vec_in = gvec_bufs[l % 2] if vec is not None else None
        if acc and vec is not None:  # the injected vec cotangent's buffer takes the gradient
            g_vec_in = injected("vec", l) if injected("vec", l) is not None else torch.zeros((N, 3, H), **o)
        flags = (nat.ACC_VEC_RESIDUAL | (nat.ACC_EDGE if l < L - 1 else 0) | meta.flags
                 | (nat.ACC_GRADS if acc else 0))
        if fused:
            kernels.et_fused_bwd_launch(qkv[:, :H], qkv[:, H:2 * H], qkv[:, 2 * H:], vec, C, u, meta.fep_imgs[l],
                                        meta.fep_frag, graph, meta.heads, g_xa, gV, g_qkv[:, :H], g_qkv[:, H:2 * H],
                                        g_qkv[:, 2 * H:], g_vec_in, g_C, g_u, g_r, accumulate=flags)
        else:
            pk = pkv[:, :H] if meta.hk else None
            pv = pkv[:, H * int(meta.hk):] if meta.hv else None
            kernels.et_message_bwd_launch(
                qkv[:, :H], qkv[:, H:2 * H], qkv[:, 2 * H:], vec, pk, pv, C, u, graph, meta.heads, g_xa, gV,
                g_qkv[:, :H], g_qkv[:, H:2 * H], g_qkv[:, 2 * H:], g_vec_in, gpk, gpv, g_C, g_u,
                accumulate=flags, pk_rows=meta.pk_rows, dpk=dpk, dpv=dpv, g_r=g_r)
        if not acc:
            if injected("qkv", l) is not None:
                g_qkv.add_(injected("qkv", l))
            if has_e and not dr and injected("pkv", l) is not None:
                g_pkv.add_(injected("pkv", l))
            if g_vec_in is not None and injected("vec", l) is not None:
                g_vec_in.add_(injected("vec", l))
        if has_e and not (meta.batched or rec) and not dr:
            if not want_f:
                pass
            elif g_f is None:
                g_f = torch.mm(g_pkv, dkv_w)
            else:
                g_f.addmm_(g_pkv, dkv_w)
        # vec_proj^T (accumulated into g_vec) and [q|k|v]^T in ONE launch
        g_xn = g_xn_all[l]
        probs = [(g_qkv, qkv_w, False, None, g_xn, False)]
        if vec is not None:
            probs.append((g_vecp.view(3 * N, 3 * H), vec_w, False, None, g_vec_in.view(3 * N, H), True))
        kernels.gemm_group(probs)
        if rec:
            step.update(g_o=g_o, g_vecp=g_vecp if vec is not None else None, g_xa=g_xa, g_qkv=g_qkv, g_xn=g_xn)
            record.append(step)
            gvec_bufs = [new((N, 3, H)), new((N, 3, H))]
        need_w = need_ws[l]
        # LayerNorm backward + residual (+ the injected x cotangent) + the previous layer's epilogue
        # backward, one kernel (with the row terms of the LayerNorm weight gradient when weights are wanted)
        prev = acts[l - 1] if l > 0 else None
        if bwd_nf and prev is not None:
            g_x, g_xa_pre = _ln_bwd_oproj(g_xn, x, mean, rstd, ln_w, gX, g_vec_in, prev[6], prev[9], layers[l - 1][9],
                                          g_vecp_all[l - 1], g_o_all[l - 1])
        else:
            g_x = _ln_bwd_epi(g_xn, x, mean, rstd, ln_w, gX, g_vec_in,
                              prev[6] if prev else None, prev[9] if prev else None,
                              g_vecp_all[l - 1] if prev else None, g_o_all[l - 1] if prev else None,
                              wrows=ln_rows[l] if any_w else None, g_res2=injected("x", l), acc=acc)
        epi_done = prev is not None
        if need_w and has_e and not (meta.batched or rec):
            base = l * meta.np
            g_w, g_b = torch.mm(g_pkv.t(), f), g_pkv.sum(0)
            if meta.planar:
                oinv = meta.perms[5]
                g_w, g_b = g_w.index_select(0, oinv), g_b.index_select(0, oinv)
            gl = _dkv_param_grads(meta, g_w, g_b)
            g_params[base + 11:base + 11 + len(gl)] = gl
        gX = g_x
        gV = g_vec_in
    adj = inj.get("W")  # the adjoint pass's weight terms (force-loss second order)
    if any_w:
        _node_weight_grads(meta, g_params, need_ws, g_qkv_all, g_o_all, g_vecp_all, g_xn_all, ln_rows, adj)
    if rec:
        record.append({"g_pkv": g_pkv_all if has_e else None, "stacks": (g_qkv_all, g_o_all, g_vecp_all),
                       "dpkv": dpkv_all if dr else None})
    if has_e and (meta.batched or rec) and not dr:  # every layer's edge-feature / projection gradients in one GEMM each
        g_f = torch.mm(g_pkv_all, meta.dkv_eff[0]) if want_f else None
        if any(need_ws[:meta.n_layers]):
            if PROJ_WGRAD == "tn":  # weight + bias (+ the adjoint's g_pkv^T gb_f): one split-K TN launch
                # (a static-capacity list: the sums stop at the device pair count, the padding rows are zero)
                g_w_all, g_b_all = kernels._linear_wgrad(g_pkv_all, f, True, True,
                                                         seg2=adj.get("dkv") if adj is not None else None,
                                                         rows=_edge_rows(meta.graph, g_pkv_all))
            else:
                g_w_all = torch.mm(g_pkv_all.t(), f)
                if adj is not None and adj.get("dkv") is not None:  # + the adjoint's g_pkv^T gb_f
                    g_w_all.addmm_(adj["dkv"][0].t(), adj["dkv"][1])
                g_b_all = g_pkv_all.sum(0)
            if meta.planar:
                dinv = meta.perms[3]
                g_w_all, g_b_all = g_w_all.index_select(0, dinv), g_b_all.index_select(0, dinv)
            for l in range(meta.n_layers):
                if need_ws[l]:
                    base = l * meta.np + 11
                    a, b = l * D, (l + 1) * D
                    gl = _dkv_param_grads(meta, g_w_all[a:b], g_b_all[a:b])
                    g_params[base:base + len(gl)] = gl
    return gX, g_f, g_C, g_u, g_r, g_params


def _edge_rows(graph, rows_tensor):
    """The device pair count of a static-capacity graph whose per-edge rows ``rows_tensor`` holds (CUDA),
    else None."""
    npd = getattr(graph, "num_pairs_dev", None)
    if npd is None or not getattr(graph, "static", False) or not rows_tensor.is_cuda \
            or rows_tensor.shape[0] != graph.n_edges:
        return None
    return npd


def _node_weight_grads(meta, g_params, need_ws, g_qkv_all, g_o_all, g_vecp_all, g_xn_all, ln_rows, adj):
    """Every layer's LayerNorm, [q|k|v], vec_proj and o_proj weight gradients at once: one batched GEMM
    per weight kind over the layer-stacked activations of the forward (meta.stk) and one reduction per
    bias (instead of ~8 launches per layer); ``adj`` (the adjoint pass's stacked factors, force-loss
    second order) is accumulated by the same batched GEMMs (baddbmm)."""
    L, N, H = meta.n_layers, g_xn_all.shape[1], meta.H
    xn_all, xa_all, vec_all = meta.stk
    if NODE_WGRAD == "tn" and g_xn_all.is_cuda and g_xn_all.dtype == torch.float32 and not meta.planar:
        return _node_weight_grads_tn(meta, g_params, need_ws, g_qkv_all, g_o_all, g_vecp_all, g_xn_all, ln_rows,
                                     adj)
    W_qkv = torch.bmm(g_qkv_all.transpose(1, 2), xn_all)
    W_o = torch.bmm(g_o_all.transpose(1, 2), xa_all)
    W_vec = torch.zeros((L, 3 * H, H), dtype=g_xn_all.dtype, device=g_xn_all.device)
    if L > 1:  # layer 0 has no vec input (vec = 0): its vec_proj gradient is zero
        torch.bmm(g_vecp_all[1:].view(L - 1, 3 * N, 3 * H).transpose(1, 2), vec_all[1:].view(L - 1, 3 * N, H),
                  out=W_vec[1:])
    W_ln = ln_rows.sum(1)
    if adj is not None:
        A, B = adj["qkv"]
        W_qkv.baddbmm_(A.transpose(1, 2), B)
        A, B = adj["o"]
        W_o.baddbmm_(A.transpose(1, 2), B)
        if adj.get("vec") is not None and L > 1:
            A, B = adj["vec"]
            W_vec[1:].baddbmm_(A[1:].view(L - 1, 3 * N, 3 * H).transpose(1, 2), B[1:].view(L - 1, 3 * N, H))
        W_ln.add_(adj["ln"].sum(1))
    B_qkv, B_o, B_ln = g_qkv_all.sum(1), g_o_all.sum(1), g_xn_all.sum(1)
    if meta.planar:  # back to the parameters' (reference) row order
        qinv = meta.perms[1]
        W_qkv, B_qkv = W_qkv.index_select(1, qinv), B_qkv.index_select(1, qinv)
    for l in range(L):
        if not need_ws[l]:
            continue
        base = l * meta.np
        wq, bq = W_qkv[l], B_qkv[l]
        g_params[base:base + 11] = [W_ln[l], B_ln[l], wq[:H], bq[:H], wq[H:2 * H], bq[H:2 * H], wq[2 * H:],
                                    bq[2 * H:], W_vec[l], W_o[l], B_o[l]]


def _node_weight_grads_tn(meta, g_params, need_ws, g_qkv_all, g_o_all, g_vecp_all, g_xn_all, ln_rows, adj):
    """_node_weight_grads as grouped TN GEMMs (tmdnet_gemm_tn_f32_ws): per layer the [q|k|v] and o_proj
    weights with their biases (the ones column, written to its own vector), vec_proj, the LayerNorm
    weight (column sums of the weight rows) and bias -- the adjoint's terms as each sum's second row
    segment -- in two launches for all layers, instead of six batched GEMMs and seven reductions."""
    L, N, H = meta.n_layers, g_xn_all.shape[1], meta.H
    xn_all, xa_all, vec_all = meta.stk
    o = dict(dtype=g_xn_all.dtype, device=g_xn_all.device)
    W_qkv, B_qkv = torch.empty((L, g_qkv_all.shape[2], H), **o), torch.empty((L, g_qkv_all.shape[2]), **o)
    W_o, B_o = torch.empty((L, g_o_all.shape[2], H), **o), torch.empty((L, g_o_all.shape[2]), **o)
    W_vec = torch.empty((L, 3 * H, H), **o)
    W_ln, B_ln = torch.empty((L, H), **o), torch.empty((L, H), **o)
    probs = []
    for l in range(L):
        if not need_ws[l]:
            continue
        seg = lambda key: {} if adj is None or adj.get(key) is None else {"A2": adj[key][0][l], "B2": adj[key][1][l]}  # noqa: E731
        probs.append({"A": g_qkv_all[l], "B": xn_all[l], "C": W_qkv[l], "Cb": B_qkv[l], "ones": True, **seg("qkv")})
        probs.append({"A": g_o_all[l], "B": xa_all[l], "C": W_o[l], "Cb": B_o[l], "ones": True, **seg("o")})
        if l > 0:
            sv = {}
            if adj is not None and adj.get("vec") is not None:
                sv = {"A2": adj["vec"][0][l].view(3 * N, 3 * H), "B2": adj["vec"][1][l].view(3 * N, H)}
            probs.append({"A": g_vecp_all[l].view(3 * N, 3 * H), "B": vec_all[l].view(3 * N, H), "C": W_vec[l], **sv})
        else:  # layer 0 has no vec input (vec = 0): its vec_proj gradient is zero
            W_vec[0].zero_()
        sl = {"A2": adj["ln"][l], "ones2": True} if adj is not None else {}
        probs.append({"A": ln_rows[l], "B": None, "C": W_ln[l].view(H, 1), "ones": True, **sl})
        probs.append({"A": g_xn_all[l], "B": None, "C": B_ln[l].view(H, 1), "ones": True})
    kernels.wgrad_tn(probs)
    for l in range(L):
        if not need_ws[l]:
            continue
        base = l * meta.np
        wq, bq = W_qkv[l], B_qkv[l]
        g_params[base:base + 11] = [W_ln[l], B_ln[l], wq[:H], bq[:H], wq[H:2 * H], bq[H:2 * H], wq[2 * H:],
                                    bq[2 * H:], W_vec[l], W_o[l], B_o[l]]


def ln_adjoint(gbar, x, mean, rstd, w, g_y):
    """VJP of the LayerNorm backward g_x = LNB(g_y, x) = rstd (a - mean(a) - xh mean(a xh)), a = g_y w
    (no residual) for the cotangent ``gbar`` of g_x.  Returns (gbar_gy, x_bar, w_bar):
      gbar_gy = w J0 gbar (J0 v = rstd (v - mean v - xh mean(v xh)), the LayerNorm Jacobian without w);
      x_bar   = -S rstd^2 xh / H - rstd/H ((a.xh) J0 gbar + (gbar.xh) J0 a),
                S = gbar.a - (sum gbar)(sum a)/H - (gbar.xh)(a.xh)/H   (row-wise sums);
      w_bar   = sum over rows of g_y * J0 gbar."""
    H = x.shape[1]
    xh = (x - mean) * rstd

    def J0(v):
        return rstd * (v - v.mean(1, keepdim=True) - xh * (v * xh).mean(1, keepdim=True))

    a = g_y * w
    Jg = J0(gbar)
    axh = (a * xh).sum(1, keepdim=True)
    gxh = (gbar * xh).sum(1, keepdim=True)
    S = (gbar * a).sum(1, keepdim=True) - gbar.sum(1, keepdim=True) * a.sum(1, keepdim=True) / H - gxh * axh / H
    x_bar = -S * rstd * rstd * xh / H - (rstd / H) * (axh * Jg + gxh * J0(a))
    return w * Jg, x_bar, (g_y * Jg).sum(0)


def epi_adjoint(gb_o, gb_vecp, gX, gV, vecp, o):
    """VJP of the epilogue backward (tmdnet_et_epilogue_bwd: g_o1 = sum_a gV v3, g_o2 = gX (v1.v2),
    g_o3 = gX, g_v1 = gX o2 v2, g_v2 = gX o2 v1, g_v3 = gV o1) for the cotangents gb_o [N, 3H],
    gb_vecp [N, 3, 3H] of its outputs.  Returns (gbar_gX, gbar_gV, vecp_bar, o_bar); vecp None (the
    first layer: vec = 0): only gbar_gX = gb_o3 is non-zero."""
    H = gX.shape[1]
    if vecp is None:
        return gb_o[:, 2 * H:], None, None, torch.zeros_like(o)
    o1, o2 = o[:, :H], o[:, H:2 * H]
    v1, v2, v3 = vecp[..., :H], vecp[..., H:2 * H], vecp[..., 2 * H:]
    b1, b2, b3 = gb_o[:, :H], gb_o[:, H:2 * H], gb_o[:, 2 * H:]
    c1, c2, c3 = gb_vecp[..., :H], gb_vecp[..., H:2 * H], gb_vecp[..., 2 * H:]
    cross = (c1 * v2 + c2 * v1).sum(1)
    gbar_gX = b2 * (v1 * v2).sum(1) + b3 + o2 * cross
    gbar_gV = b1.unsqueeze(1) * v3 + c3 * o1.unsqueeze(1)
    gxo2 = (gX * o2).unsqueeze(1)
    bgx = (b2 * gX).unsqueeze(1)
    vecp_bar = torch.cat((bgx * v2 + c2 * gxo2, bgx * v1 + c1 * gxo2, b1.unsqueeze(1) * gV), dim=-1)
    o_bar = torch.cat(((c3 * gV).sum(1), gX * cross, torch.zeros_like(gX)), dim=1)
    return gbar_gX, gbar_gV, vecp_bar, o_bar


def adjoint_epi_ln_launch(epi, gbar_x_in, gbar_vec_in, ln, outs=None):
    """One ``tmdnet_et_adjoint_epi_ln`` launch: layer l's epilogue-backward VJP (``epi`` = (gb_o,
    gb_vecp, gX, gV, vecp, o) or None) fused with the next LayerNorm-backward VJP (``ln`` = (x, mean,
    rstd, ln_w, g_y) or None).  Returns (gbar_x_out, gbar_vec_out, vecp_bar, o_bar, gbar_gy, x_bar,
    w_bar) with w_bar the weight cotangent (column sum of the kernel's per-row products).  The Python
    ``epi_adjoint`` / ``ln_adjoint`` restate it (CPU tests).  ``outs`` (optional dict): caller buffers
    "gbgy" (gbar_gy), "gbv" (gbar_vec_out), "wrows" (the per-row weight terms: w_bar is then None and
    the caller sums the rows).  ``gbar_vec_in`` may be a pair (a, b): the cotangent a + b, summed by the
    kernel (tmdnet_et_adjoint_epi_ln2)."""
    lib = nat.load()
    outs = outs or {}
    N, H = gbar_x_in.shape
    gbar_vec_in2 = None
    if isinstance(gbar_vec_in, tuple):
        gbar_vec_in, gbar_vec_in2 = gbar_vec_in
    o_ = dict(dtype=gbar_x_in.dtype, device=gbar_x_in.device)
    gb_o = gb_vecp = gX = gV = vecp = o = None
    gbx_out = gbv_out = vpbar = obar = None
    if epi is not None:
        gb_o, gb_vecp, gX, gV, vecp, o = epi
        gbx_out = torch.empty((N, H), **o_)
        obar = outs["obar"] if outs.get("obar") is not None else torch.empty((N, 3 * H), **o_)
        if vecp is not None or gbar_vec_in is not None or gbar_vec_in2 is not None:
            gbv_out = outs["gbv"] if outs.get("gbv") is not None else torch.empty((N, 3, H), **o_)
        if vecp is not None:
            vpbar = outs["vpbar"] if outs.get("vpbar") is not None else torch.empty((N, 3, 3 * H), **o_)
    x = mean = rstd = w = gy = gbgy = xbar = wrows = None
    if ln is not None:
        x, mean, rstd, w, gy = ln
        gbgy = outs["gbgy"] if outs.get("gbgy") is not None else torch.empty((N, H), **o_)
        wrows = outs["wrows"] if outs.get("wrows") is not None else torch.empty((N, H), **o_)
        xbar = torch.empty((N, H), **o_)
    c = lambda t: None if t is None else t.contiguous()  # noqa: E731
    args = [c(t) for t in (gb_o, gb_vecp, gX, gV, vecp, o, gbar_x_in, gbar_vec_in, gbar_vec_in2)]
    rc = lib.tmdnet_et_adjoint_epi_ln2(nat.dtype_code(gbar_x_in.dtype), N, H, *[nat.ptr(t) for t in args],
                                       nat.ptr(gbx_out), nat.ptr(gbv_out), nat.ptr(vpbar), nat.ptr(obar),
                                       *[nat.ptr(c(t)) for t in (x, mean, rstd, w, gy)], nat.ptr(gbgy),
                                       nat.ptr(xbar), nat.ptr(wrows), nat.stream(gbar_x_in.device))
    nat.check(rc, "tmdnet_et_adjoint_epi_ln2")
    if epi is None:
        gbx_out = gbar_x_in
        gbv_out = gbar_vec_in if gbar_vec_in2 is None else \
            (gbar_vec_in2 if gbar_vec_in is None else gbar_vec_in + gbar_vec_in2)
    # (the column sums as a split-K TN launch: ATen's dim-0 reduction of [N, H] took 20 us at C2)
    return gbx_out, gbv_out, vpbar, obar, gbgy, xbar, \
        (kernels._linear_wgrad(wrows, wrows, False, True)[1] if (wrows is not None and outs.get("wrows") is None)
         else None)


def adjoint_epi_ln_composite(epi, gbar_x_in, gbar_vec_in, ln, outs=None):
    """``adjoint_epi_ln_launch`` restated with ``epi_adjoint`` / ``ln_adjoint`` (CPU tests)."""
    if isinstance(gbar_vec_in, tuple):  # (a, b): the cotangent a + b
        a, b = gbar_vec_in
        gbar_vec_in = b if a is None else (a if b is None else a + b)
    if outs:
        res = list(adjoint_epi_ln_composite(epi, gbar_x_in, gbar_vec_in, ln))
        if outs.get("gbv") is not None and res[1] is not None:
            outs["gbv"].copy_(res[1])
            res[1] = outs["gbv"]
        if outs.get("obar") is not None and res[3] is not None:
            outs["obar"].copy_(res[3])
            res[3] = outs["obar"]
        if outs.get("vpbar") is not None and res[2] is not None:
            outs["vpbar"].copy_(res[2])
            res[2] = outs["vpbar"]
        if outs.get("gbgy") is not None and res[4] is not None:
            outs["gbgy"].copy_(res[4])
            res[4] = outs["gbgy"]
        if outs.get("wrows") is not None and ln is not None:
            x, mean, rstd, w, gy = ln
            xh = (x - mean) * rstd
            J0 = lambda v: rstd * (v - v.mean(1, keepdim=True) - xh * (v * xh).mean(1, keepdim=True))  # noqa: E731
            outs["wrows"].copy_(gy * J0(res[0]))
            res[6] = None
        return tuple(res)
    gbx, gbv, vpbar, obar = gbar_x_in, gbar_vec_in, None, None
    if epi is not None:
        e_x, e_v, vpbar, obar = epi_adjoint(*epi)
        gbx = gbar_x_in + e_x
        if e_v is not None:
            gbv = e_v if gbar_vec_in is None else gbar_vec_in + e_v
    gbgy = xbar = wb = None
    if ln is not None:
        x, mean, rstd, w, gy = ln
        gbgy, xbar, wb = ln_adjoint(gbx, x, mean, rstd, w, gy)
    return gbx, gbv, vpbar, obar, gbgy, xbar, wb


def hand_second_order_ok(meta, dr, need_w, ggs_params):
    """The hand-scheduled second order covers the force-pass node (no weight gradients in its
    outputs) in the reference row layout; otherwise the composite recompute runs."""
    return (not meta.planar and not any(need_w) and all(g is None for g in ggs_params)
            and (not dr or meta.rbf is not None))


def _second_order(ctx, ggs, want):
    """Hand-scheduled second order of the force pass (the VJP of _backward_layers for the cotangents
    ``ggs`` of its outputs g_x, g_f, g_C, g_u, g_r), replacing autograd's double differentiation of
    the recomputed stack (~2.6k small kernels per ET-QM9 training step).  Three passes:

    1. re-run the first-order backward without dr mode, recording every layer's intermediates
       (seeds, g_o, g_vecp, g_xa, g_qkv, g_xn, the per-edge projection gradient);
    2. the ADJOINT of that backward, in forward layer order: per layer the LayerNorm-backward VJP
       (``ln_adjoint``), the two node GEMMs' transposes, the message backward's VJP
       (tmdnet_et_message_bwd2, HIP), the o-GEMM transpose and the epilogue-backward VJP
       (``epi_adjoint``).  It yields the cotangents of the seeds gX / gV (returned), of the weights
       the backward multiplies by, and of every forward intermediate (x, vec, [q|k|v], projection,
       vecp, o);
    3. one more first-order backward through the forward layers with those intermediate cotangents
       injected where the backward forms their gradients (``inject``), giving the gradients of the
       stack's inputs and weights.

    ``want`` (per saved input gX, gV, x, f, C, u, r, *params): which gradients the engine consumes."""
    saved = ctx.saved_tensors
    gX, gV, x, f, C, u, r = saved[:7]
    params = list(saved[7:])
    meta = ctx.meta
    acts = ctx.acts
    L, H, D = meta.n_layers, meta.H, meta.D
    N, E = x.shape[0], meta.graph.n_edges
    graph = meta.graph
    o = dict(dtype=x.dtype, device=x.device)
    has_e = bool(meta.hk or meta.hv)
    gg_x, gg_f, gg_C, gg_u, gg_r = ggs[:5]
    layers = meta.split(params)
    need_none = (False,) * (L + int(meta.out_norm))
    # 1. the force pass recorded: by the force pass itself when it ran under create_graph (ctx.rec),
    # else again here (its outputs are those of the dr-mode pass up to round-off)
    rec, g_f0 = getattr(ctx, "rec", None), getattr(ctx, "g_f0", None)
    ctx.rec = ctx.g_f0 = None
    if rec is None:
        rec = []
        _, g_f0, _, _, _, _ = _backward_layers(meta, gX, gV, f, C, u, params, acts, need_none, record=rec,
                                               want_f=bool(want[6]))  # g_f0: only for d/dr of g_r
    tail = rec.pop()
    g_pkv_all = tail["g_pkv"] if has_e else None
    rg_qkv_all, rg_o_all, rg_vecp_all = tail["stacks"]
    rec = rec[::-1]  # layer 0 first
    W_all = meta.dkv_eff[0]
    if g_f0 is None and want[6] and has_e:  # (the recorded dr pass does not form g_f)
        g_f0 = torch.mm(g_pkv_all, W_all)
    # cotangent of the summed edge-feature gradient g_f = g_pkv_all W_all
    gb_f = gg_f
    r_bar = None
    if ctx.dr and gg_r is not None and has_e:
        fdp = kernels.rbf_deriv(r, *meta.rbf)
        gb_r_f = gg_r.unsqueeze(1) * fdp
        gb_f = gb_r_f if gb_f is None else gb_f + gb_r_f
        if want[6]:  # d/dr of g_r = <g_f, df/dr>: the RBF's second derivative (composite)
            with torch.enable_grad():
                rr = r.detach().requires_grad_(True)
                fd, = torch.autograd.grad(kernels.rbf_composite(rr, *meta.rbf), rr, g_f0.detach(),
                                          create_graph=True)
                r_bar, = torch.autograd.grad(fd, rr, gg_r)
    # the projection rows' cotangent gb_f W^T: with only the g_r term (gg_f None) it is gg_r[e] times the
    # pair rows' d(dk,dv)/dr the recorded dr pass formed -- the message VJP scales those rows per edge
    # (no E x layers*D product); otherwise one GEMM
    dpkv_pairs = tail.get("dpkv") if (gg_f is None and ctx.dr and gg_r is not None and meta.pk_rows is not None) else None
    gb_pkv_all = None
    if dpkv_pairs is None and gb_f is not None and has_e:
        gb_pkv_all = meta.dkv_proj(gb_f, bias=False)
    gr_scale = gg_r.contiguous() if dpkv_pairs is not None else None
    W_bar = {}

    def acc(key, val):
        W_bar[key] = val if key not in W_bar else W_bar[key] + val

    inj = {k: [None] * L for k in ("o", "vecp", "qkv", "pkv", "vec", "x")}
    # the weight cotangents of the backward's node GEMMs / LayerNorms are formed batched over layers by
    # pass 3 (_node_weight_grads): here only their factors, stacked per layer
    gbgxn_all, dgxa_all, wrows_all = (torch.empty((L, N, H), **o) for _ in range(3))
    gbv_all = torch.empty((L, N, 3, H), **o)
    # the injections themselves, layer-stacked: pass 3's kernels accumulate into these buffers
    inj["stk"] = {"qkv": torch.empty((L, N, 5 * H), **o), "o": torch.empty((L, N, 3 * H), **o),
                  "vecp": torch.empty((L, N, 3, 3 * H), **o),
                  "pkv": torch.empty((E, L * D), **o) if has_e else None}
    inj["W"] = {"qkv": (rg_qkv_all, gbgxn_all), "o": (rg_o_all, dgxa_all), "vec": (rg_vecp_all, gbv_all),
                "ln": wrows_all, "dkv": None}
    if gb_f is not None and has_e:
        if meta.batched:
            inj["W"]["dkv"] = (g_pkv_all, gb_f)  # accumulated into pass 3's edge-feature weight GEMM
        else:
            acc("dkv", torch.mm(g_pkv_all.t(), gb_f))
    C_bar = torch.empty((E,), **o)  # overwritten by layer 0's message VJP, accumulated by the others
    u_bar = torch.empty((E, 3), **o)
    gbar_x = gg_x if gg_x is not None else torch.zeros((N, H), **o)
    gbar_v = None
    ggC = gg_C if gg_C is not None else torch.zeros((E,), **o)
    ggu = gg_u if gg_u is not None else torch.zeros((E, 3), **o)

    def ln_of(l):  # the LayerNorm whose backward-VJP follows layer l-1's epilogue VJP
        if l < L:
            a = acts[l]
            return (a[0], a[3], a[4], layers[l][0], rec[l]["g_xn"])
        if meta.out_norm:
            x_pre, mean_o, rstd_o = acts[L]
            return (x_pre, mean_o, rstd_o, params[-2], gX)
        return None

    # 2. the adjoint pass, layer 0 first (layer 0's LayerNorm VJP alone, then per layer the node GEMM
    # transposes, the message VJP and the fused epilogue VJP + next LayerNorm VJP)
    _, _, _, _, gb_gxn, inj["x"][0], _ = adjoint_epi_ln_launch(None, gbar_x, None, ln_of(0),
                                                                outs={"gbgy": gbgxn_all[0], "wrows": wrows_all[0]})
    seed_x = None
    on_bar = None
    for l in range(L):
        p = layers[l]
        R = rec[l]
        x_l, vec_l, xn, mean, rstd, qkv, vecp, pkv, xa, o_ = _act_pkv(meta, acts, l, f)
        vec_w, o_w = p[8], p[9]
        qkv_w = meta.qkv_eff[l][0]
        # the two input-side transposes in one grouped launch: gb_gqkv = gb_gxn qkv_w^T, gb_gvecp =
        # gbar_v vec_w^T
        gb_gqkv = torch.empty((N, qkv_w.shape[0]), **o)
        probs = [(gb_gxn, qkv_w, True, None, gb_gqkv, False)]
        gb_gvecp = None
        if vec_l is not None and gbar_v is not None:
            gb_gvecp = torch.empty((N, 3, 3 * H), **o)
            probs.append((gbar_v.reshape(3 * N, H), vec_w, True, None, gb_gvecp.view(3 * N, 3 * H), False))
        elif l > 0:  # no vec cotangent reached this layer: its vec_proj weight term is zero
            gbv_all[l].zero_()
        kernels.gemm_group(probs)
        # message backward VJP (per-edge projection rows)
        pk = pv = None
        if has_e:  # the pair-shared projection rows, read through pk_rows by the kernel
            pk = pkv[:, :H] if meta.hk else None
            pv = pkv[:, H * int(meta.hk):] if meta.hv else None
        gbl = gb_pkv_all[:, l * D:(l + 1) * D] if gb_pkv_all is not None else None
        if dpkv_pairs is not None:
            gbl = dpkv_pairs[:, l * D:(l + 1) * D]
        ggs_m = (gb_gqkv[:, :H], gb_gqkv[:, H:2 * H], gb_gqkv[:, 2 * H:],
                 gbar_v if vec_l is not None else None,
                 gbl[:, :H] if (gbl is not None and meta.hk) else None,
                 gbl[:, H * int(meta.hk):] if (gbl is not None and meta.hv) else None, ggC, ggu)
        # d_q | d_k | d_v and d_pk | d_pv written straight into the injection buffers, the cutoff /
        # unit-vector cotangents accumulated into C_bar / u_bar by the kernel
        outs = {"qkv": inj["stk"]["qkv"][l], "C": C_bar, "u": u_bar, "gx": dgxa_all[l], "edge_overwrite": l == 0}
        if has_e:
            outs["pkv"] = inj["stk"]["pkv"][:, l * D:(l + 1) * D]
        d_gxa, d_gvec, d_q, d_k, d_v, d_vec, d_pk, d_pv, d_C, d_u = kernels.et_message_bwd2_launch(
            qkv[:, :H], qkv[:, H:2 * H], qkv[:, 2 * H:], vec_l, pk, pv, C, u, graph, meta.heads,
            R["g_xa"], R["gV"] if R["gV"] is not None else torch.zeros((N, 3, H), **o), ggs_m, out=outs,
            pk_rows=meta.pk_rows if has_e else None, gg_pkv_scale=gr_scale, flags=meta.acts)
        inj["qkv"][l] = outs["qkv"]
        if has_e:
            inj["pkv"][l] = outs["pkv"]
        inj["vec"][l] = d_vec
        # the vec residual g_vec = gV + ...: the two addends go to the adjoint kernel, which sums them on load
        gb_gV = d_gvec if gbar_v is None else (gbar_v, d_gvec)
        gb_go = torch.empty((N, o_w.shape[0]), **o)
        kernels.gemm_group([(d_gxa, o_w, True, None, gb_go, False)])
        if gb_gvecp is None and vecp is not None:
            gb_gvecp = torch.zeros((N, 3, 3 * H), **o)
        nxt = ln_of(l + 1)
        nx = {"gbgy": gbgxn_all[l + 1], "gbv": gbv_all[l + 1], "wrows": wrows_all[l + 1]} if l + 1 < L else {}
        nx["obar"] = inj["stk"]["o"][l]
        nx["vpbar"] = inj["stk"]["vecp"][l]
        gbar_x, gbar_v, inj["vecp"][l], inj["o"][l], gb_gxn, xb, wb = adjoint_epi_ln_launch(
            (gb_go, gb_gvecp, R["gX"], R["gV"], vecp, o_), gbar_x, gb_gV, nxt, outs=nx)
        if l + 1 < L:
            inj["x"][l + 1] = xb
        elif nxt is not None:  # the fused out_norm: its input's cotangent seeds pass 3
            seed_x, on_bar = xb, wb
            gbar_x = gb_gxn
    # 3. the backward through the forward layers with the injected cotangents.  When the forward
    # node's own backward runs later in this same pass (training: the energy loss and the head's
    # second order reach it), the injections are handed to it (meta.pending) and it runs ONE
    # backward for both -- no second pass, and no engine-side sums of two parameter gradients.
    ref = getattr(meta, "fwd_node", None)
    node = ref() if ref is not None else None
    if node is not None and _will_run(node):
        inj["x_top"] = seed_x
        meta.pending = {"inj": inj, "W_bar": W_bar, "on_bar": on_bar, "C_bar": C_bar, "u_bar": u_bar}
        # prune entries that are gone or already consumed (custom loops never call check_pending_consumed)
        _HANDED_OFF[:] = [r for r in _HANDED_OFF if (m := r()) is not None and getattr(m, "pending", None) is not None]
        _HANDED_OFF.append(weakref.ref(meta))
        res = [gbar_x, gbar_v, None, None, None, None, r_bar] + [None] * len(params)
        return [t if w else None for t, w in zip(res, want)]
    need_w = tuple(bool(w) for w in _layer_wants(meta, want[7:]))
    g_x, g_f, g_C, g_u, _, g_params = _backward_layers(
        meta, seed_x if seed_x is not None else torch.zeros((N, H), **o), torch.zeros((N, 3, H), **o),
        f, C, u, params, acts, need_w, inject=inj, seed_pre_norm=meta.out_norm)
    g_C = g_C + C_bar
    g_u = g_u + u_bar
    g_params = _apply_w_bar(meta, list(g_params), W_bar, on_bar, lambda i: want[7 + i])
    res = [gbar_x, gbar_v, g_x, g_f, g_C, g_u, r_bar] + g_params
    return [t if w else None for t, w in zip(res, want)]


def _apply_w_bar(meta, g_params, W_bar, on_bar, wanted):
    """Add the adjoint pass's weight cotangents (the weights the first-order backward multiplies by:
    LayerNorm weights, [q|k|v], vec_proj, o_proj, dk/dv, out_norm) to the parameters' gradients."""
    H, D = meta.H, meta.D

    def addp(i, val):
        if val is not None and wanted(i):
            g_params[i] = val if g_params[i] is None else g_params[i] + val

    for l in range(meta.n_layers):  # (the node weights' terms are added by _node_weight_grads)
        base = l * meta.np
        if "dkv" in W_bar:
            wl = W_bar["dkv"][l * D:(l + 1) * D]
            for j, gw in enumerate(_dkv_param_grads(meta, wl, wl[:, 0])[0::2]):
                addp(base + 11 + 2 * j, gw)
    if on_bar is not None:
        addp(len(g_params) - 2, on_bar)
    return g_params


def _layer_wants(meta, want_params):
    """Per-layer (and out_norm) weight-gradient request from the per-parameter ``want`` flags."""
    out = [any(want_params[l * meta.np:(l + 1) * meta.np]) for l in range(meta.n_layers)]
    if meta.out_norm:
        out.append(any(want_params[-2:]))
    return out


def _dkv_param_grads(meta, g_w, g_b):
    """[dk_w, dk_b, dv_w, dv_b] (those present) from one layer's [dk; dv] gradient rows."""
    H = meta.H
    out = []
    if meta.hk:
        out += [g_w[:H], g_b[:H]]
    if meta.hv:
        a = H * int(meta.hk)
        out += [g_w[a:], g_b[a:]]
    return out


def composite_stack(meta, x, f, C, u, params, message=None):
    """Reference math (torchmd_et.py:177-184, 293-321) as differentiable ops.  ``message`` is the
    ET message implementation: the HIP autograd Functions (``kernels.et_message``, whose backward
    and second-order backward are HIP kernels) or, by default, the plain PyTorch restatement."""
    H = meta.H
    graph = meta.graph
    src, dst = graph.src.long(), graph.dst.long()
    N = x.shape[0]
    vec = torch.zeros((N, 3, H), dtype=x.dtype, device=x.device)
    layers = meta.split(params)
    D = meta.D
    # every layer's dk/dv projection as ONE GEMM (differentiable cat of the parameters): one
    # weight-gradient GEMM over the E rows instead of one per layer and projection
    # splits, not slices: a split's backward is ONE cat of the pieces' gradients, where every slice's
    # backward zero-fills a tensor of the whole size and autograd then adds them up (this graph is
    # differentiated twice by the second order, so each saved launch counts twice)
    pkv_layers = None
    if D:
        rest = [p[11:] for p in layers]
        w_all = torch.cat([w for r in rest for w in r[0::2]], 0)
        b_all = torch.cat([b for r in rest for b in r[1::2]], 0)
        pkv_layers = torch.split(F.linear(f, w_all, b_all), D, dim=1)
    for l, p in enumerate(layers):
        ln_w, ln_b, q_w, q_b, k_w, k_b, v_w, v_b, vec_w, o_w, o_b = p[:11]
        xn = F.layer_norm(x, (H,), ln_w, ln_b, _EPS)
        # [q|k|v] as one product (three GEMMs fewer in each of the three passes over this graph)
        q, k, v = torch.split(F.linear(xn, torch.cat((q_w, k_w, v_w)), torch.cat((q_b, k_b, v_b))),
                              [q_w.shape[0], k_w.shape[0], v_w.shape[0]], dim=1)
        vec1, vec2, vec3 = torch.split(F.linear(vec, vec_w), H, dim=-1)
        vec_dot = (vec1 * vec2).sum(dim=1)
        pk = pv = None
        if D:
            hk_w = H * int(meta.hk)
            pk, pv = torch.split(pkv_layers[l], [hk_w, D - hk_w], dim=1)
            pk = pk if meta.hk else None
            pv = pv if meta.hv else None
        if message is None:
            xa, veca = kernels.et_message_composite(q, k, v, vec, pk, pv, C, u, src, dst, N, meta.heads, meta.acts)
        else:
            xa, veca = message(q, k, v, vec, pk, pv, C, u)
        o1, o2, o3 = torch.split(F.linear(xa, o_w, o_b), H, dim=1)
        x = x + vec_dot * o2 + o3
        vec = vec + vec3 * o1.unsqueeze(1) + veca
    if meta.out_norm:
        x = F.layer_norm(x, (H,), params[-2], params[-1], _EPS)
    return x, vec


# stacks whose second order handed its injected cotangents to the forward node's backward
# (meta.pending); check_pending_consumed() after the loss backward proves they were all taken
_HANDED_OFF = []


def check_pending_consumed():
    """Raise if a second order's injected cotangents were handed to a forward node whose backward then
    never ran in the same engine pass (its parameter gradients would silently lack those terms)."""
    left = [m for m in (ref() for ref in _HANDED_OFF) if m is not None and getattr(m, "pending", None) is not None]
    _HANDED_OFF.clear()
    for m in left:
        m.pending = None
    if kernels.head_pending_left():
        raise RuntimeError("torchmd-net_amd: the output head's second-order weight terms were not consumed by "
                           "the head's backward (engine order); the parameter gradients are incomplete")
    if left:
        raise RuntimeError("torchmd-net_amd: the ET stack's second-order cotangents were not consumed by the "
                           "forward node's backward (engine order); the parameter gradients are incomplete")


def _will_run(node):
    if node is None:  # parameter without requires_grad
        return False
    try:
        return bool(torch._C._will_engine_execute_node(node))
    except RuntimeError:
        return True


class _ETStack(Function):
    @staticmethod
    def forward(ctx, meta, x, f, C, u, r, *params):
        # (autograd is off inside forward: whether a backward can follow is the caller's grad mode and
        # what the inputs say -- needs_input_grad alone follows requires_grad, also under no_grad)
        want = meta.grad_mode and any(ctx.needs_input_grad)
        x_out, vec_out, acts = _forward_layers(meta, x, f, C, u, params, r=r, want_bwd=want)
        ctx.meta = meta
        ctx.acts = acts
        meta.fwd_node = weakref.ref(ctx)  # the second order hands its injections to this node's backward
        meta.pending = None
        ctx.save_for_backward(x, f, C, u, r, *params)
        return x_out, vec_out

    @staticmethod
    def backward(ctx, gX, gV):
        x, f, C, u, r, *params = ctx.saved_tensors
        meta = ctx.meta
        # which layers' weight gradients does THIS backward deliver?  The parameters' AccumulateGrad
        # nodes are this node's own last next edges; nothing is cached across
        # iterations -- an AccumulateGrad node kept alive from an earlier step stays bound to the
        # stream it was created on and breaks HIP-graph capture of later steps.
        nf = ctx.next_functions  # one entry per tensor argument (a None edge-feature input has none)
        off = len(nf) - len(params)
        need_w = tuple(any(_will_run(nf[off + l * meta.np + j][0]) for j in range(meta.np))
                       for l in range(meta.n_layers))
        if meta.out_norm:  # one more entry: the fused out_norm's weight / bias
            base = off + meta.n_layers * meta.np
            need_w += (_will_run(nf[base][0]) or _will_run(nf[base + 1][0]),)
        if gX is None:
            gX = torch.zeros_like(x)
        if gV is None:
            gV = torch.zeros((x.shape[0], 3, meta.H), dtype=x.dtype, device=x.device)
        # dr mode: the distances (not the features) take the edge-feature gradient -- only when no
        # weight gradient needs the projection gradient (the force pass)
        pending, meta.pending = getattr(meta, "pending", None), None
        dr = bool(meta.rbf is not None and ctx.needs_input_grad[5] and meta.D and not any(need_w))
        if DR_MODE in ("0", "off") or pending is not None:
            dr = False
        # the edge-feature gradient only when something consumes it (never in a parameter backward)
        want_f = f is not None and ctx.needs_input_grad[2] and _will_run(nf[1][0])
        if pending is not None:  # does anything consume the cutoff / unit-vector gradients (2 adds)?
            ti = [i for i, t in zip(range(2, 7), (f, C, u, r)) if t is not None]  # (x is always present)
            idx = {i: 1 + j for j, i in enumerate(ti)}
            pending["want_cu"] = any(ctx.needs_input_grad[i] and _will_run(nf[idx[i]][0]) for i in (3, 4)
                                     if i in idx)
        # a force pass whose own backward will be taken (create_graph: force-matching training) records
        # its intermediates for the hand second order right here, instead of the second order re-running
        # it: the training form (projection gradient materialised) with g_r = <g_f, df/dr> per edge
        record = (dr and torch.is_grad_enabled() and _EXPECT_SECOND_ORDER[0] and SECOND_ORDER != "composite"
                  and RECORD_IN_FORCE_PASS and hand_second_order_ok(meta, dr, need_w, ()))
        outs = _ETStackBwd.apply(meta, ctx.acts, need_w, dr, pending, want_f, record, gX.contiguous(),
                                 gV.contiguous(), x, f, C, u, r, *params)
        g_x, g_f, g_C, g_u, g_r = outs[:5]
        return (None, g_x, g_f, g_C, g_u, g_r) + tuple(outs[5:])


class _ETStackBwd(Function):
    @staticmethod
    def forward(ctx, meta, acts, need_w, dr, pending, want_f, record, gX, gV, x, f, C, u, r, *params):
        if not meta.graph.symmetric:
            raise RuntimeError("torchmd-net_amd: the ET backward source pass needs a symmetric edge "
                               "list (include_transpose=True, no capacity overflow)")
        ctx.rec = None
        if record:  # dr mode, recorded: g_r in-kernel and the projection gradient kept (_ETStack.backward)
            rec = []
            g_x, g_f, g_C, g_u, g_r, g_params = _backward_layers(meta, gX, gV, f, C, u, params, acts, need_w,
                                                                 r=r, dr=True, record=rec, want_f=False)
            ctx.rec, ctx.g_f0 = rec, None
        else:
            g_x, g_f, g_C, g_u, g_r, g_params = _backward_layers(meta, gX, gV, f, C, u, params, acts, need_w,
                                                                 r=r, dr=dr,
                                                                 inject=pending["inj"] if pending else None,
                                                                 want_f=want_f)
        if pending is not None:  # the second order's contributions (et_stack._second_order)
            if pending.get("want_cu", True):
                g_C = g_C + pending["C_bar"]
                g_u = g_u + pending["u_bar"]
            else:  # nothing downstream consumes them (a training step's parameter backward)
                g_C = g_u = None
            wl = list(need_w)
            g_params = _apply_w_bar(meta, list(g_params), pending["W_bar"], pending["on_bar"],
                                    lambda i: wl[min(i // meta.np, len(wl) - 1)] if i < meta.n_layers * meta.np
                                    else wl[-1])
        ctx.meta = meta
        ctx.dr = dr
        ctx.acts = acts
        ctx.need_w = need_w
        ctx.save_for_backward(gX, gV, x, f, C, u, r, *params)
        return (g_x, g_f, g_C, g_u, g_r) + tuple(g_params)

    @staticmethod
    def backward(ctx, *ggs):
        """Second order (force-matching training): the layers are re-run with the HIP message
        Functions and differentiated twice, so the message's second order runs the HIP kernel
        tmdnet_et_message_bwd2 and the node ops PyTorch's GEMM / layer-norm double backwards.  In dr
        mode the features are re-formed from r by the differentiable basis (the first-order output
        was g_r, so the second order must see f's dependence on r)."""
        saved = ctx.saved_tensors
        meta = ctx.meta
        graph, heads = meta.graph, meta.heads

        def message(q, k, v, vec, pk, pv, C_, u_):
            return kernels.et_message(q, k, v, vec, pk, pv, C_, u_, graph, heads, meta.acts)

        _create = torch.is_grad_enabled()  # third order only if the caller builds a graph
        n_out = 7 + len(saved)
        # inputs whose gradient this backward must deliver: asked for AND consumed downstream (a
        # training step's loss.backward(inputs=params) never runs the position branch, so the
        # cutoff / unit-vector / distance gradients -- E-sized work -- are skipped)
        nf = iter(ctx.next_functions)  # one entry per tensor argument (None arguments have none)
        want = []
        for i, t in enumerate(saved):
            node = next(nf)[0] if t is not None else None
            want.append(t is not None and ctx.needs_input_grad[7 + i] and _will_run(node))
        if SECOND_ORDER != "composite" and not _create and hand_second_order_ok(meta, ctx.dr, ctx.need_w, ggs[5:]):
            if not any(want):
                return (None,) * n_out
            return (None,) * 7 + tuple(_second_order(ctx, ggs, want))
        with torch.enable_grad():
            leaves = [None if t is None else t.detach().requires_grad_(True) for t in saved]
            gX, gV, x, f, C, u, r = leaves[:7]
            params = leaves[7:]
            f_in = kernels.rbf_composite(r, *meta.rbf) if ctx.dr else f
            xo, vo = composite_stack(meta, x, f_in, C, u, params, message=message)
            wrt = [x, f, C, u, r] + params
            # first-order gradients only for the outputs that received a cotangent (the force pass's
            # parameter gradients are never formed: their cotangents are None)
            pick = [i for i, (t, g) in enumerate(zip(wrt, ggs)) if t is not None and g is not None]
            ins = [t for t, w in zip(leaves, want) if w]
            if not pick or not ins:
                return (None,) * n_out
            first = torch.autograd.grad((xo, vo), [wrt[i] for i in pick], (gX, gV), create_graph=True,
                                        allow_unused=True)
            sel = [(fg, ggs[i]) for fg, i in zip(first, pick) if fg is not None]
            if not sel:
                return (None,) * n_out
            second = torch.autograd.grad([fg for fg, _ in sel], ins, [g for _, g in sel],
                                         create_graph=_create, allow_unused=True)
        it = iter(second)
        res = [next(it) if w else None for w in want]
        return (None,) * 7 + tuple(res)


def stack_parameters(layers):
    """Make every layer's [q|k|v] weights / biases and all layers' [dk; dv] weights / biases row blocks of
    shared buffers (``_stack_views``; no-op when they already are).  Returns (dkv_w, dkv_b, [(qkv_w, qkv_b)]).
    The C++ ``tmdnet::et_stack`` / ``et_energy_forces`` operators then take these blocks as views of the
    parameters' own storage (torch_ops.cpp ``pack_stack``): nothing is packed or cached, so optimizer steps
    and ``p.data`` writes are seen on the next call."""
    sw = getattr(layers, "_tmd_stack", None)
    if sw is None or sw.layers is not layers:
        sw = StackWeights(layers)
        layers._tmd_stack = sw
    dkv_w, dkv_b = sw.dkv()
    fused = []
    for layer in layers:
        if layer._stacked is None:
            layer._stacked = LayerWeights(layer)
        fused.append(layer._stacked.fused())
    return dkv_w, dkv_b, fused


def et_stack(layers, x, graph, f, C, u, rbf=None, out_norm=None, f_pairs=None, fdp_pairs=None):
    """Run ``layers`` (EquivariantMultiHeadAttention modules) as one node.  Returns (x, vec) after
    the last residual update (reference torchmd_et.py:180-184).

    ``rbf`` = (r, mu, beta, cutoff_lower, cutoff_upper, rbf_type) declares f = rbf(r) with a fixed
    (non-trainable) basis, which lets the force pass take its edge gradient straight to r ("dr mode",
    _backward_layers).  ``out_norm`` (nn.LayerNorm(H), the model's final norm) is applied to x inside
    the last layer's epilogue kernel.  ``f_pairs`` = f at the graph's pair rows (``pair_index``
    numbering), when already produced with f (tmdnet_edge_geom_fwd_rows); else gathered here."""
    l0 = layers[0]
    H, heads = l0.hidden_channels, l0.num_heads
    hk, hv = l0.dk_proj is not None, l0.dv_proj is not None
    params = []
    dkv_w, dkv_b, fused = stack_parameters(layers)
    for layer in layers:
        layer._check_supported()
        params += layer_params(layer)
    D = (int(hk) + 3 * int(hv)) * H
    batched = D > 0 and graph.n_edges * len(layers) * D * x.element_size() <= BATCH_DKV_BYTES
    meta = _Meta(graph, heads, H, hk, hv, len(layers), fused, None, dkv_w, dkv_b, batched)
    meta.acts = l0.act_flags  # the activations (every layer of a model shares them)
    if any(layer.act_flags != meta.acts for layer in layers):
        raise NotImplementedError("et_stack: layers with different activations")
    meta.flags = meta.acts
    if graph.n_edges >= PLANAR_MIN_EDGES:
        meta.planar, meta.flags = True, nat.ET_V_PLANAR | meta.acts
        meta.perms = _planar_perms(meta, x.device)
    if D and PAIR_ROWS and graph.symmetric and graph.transpose is not None:
        meta.pairs = kernels.pair_index(graph)
        meta.pk_rows = meta.pairs[0]
        if f_pairs is not None and f_pairs.shape[0] == meta.pairs[1].shape[0]:
            meta.f_pairs = f_pairs.detach()
            if fdp_pairs is not None and fdp_pairs.shape == f_pairs.shape:
                meta.fdp_pairs = fdp_pairs.detach()
    if out_norm is not None:
        if not (out_norm.elementwise_affine and tuple(out_norm.normalized_shape) == (H,) and out_norm.eps == _EPS):
            raise ValueError("et_stack: out_norm must be an affine nn.LayerNorm(H) with eps 1e-5")
        meta.out_norm = True
        params += [out_norm.weight, out_norm.bias]
    r = None
    if rbf is not None and D:
        r, mu, beta, cl, cu, rbf_type = rbf
        meta.rbf = (mu.detach(), beta.detach(), float(cl), float(cu), int(rbf_type))
        meta.fep = (FEP not in ("0", "off") and graph.n_edges >= FEP_MIN_EDGES and hk and hv and x.is_cuda
                    and meta.acts == 0
                    and kernels.fep_supported(H, heads, mu.shape[0], x.dtype) and r.dtype == x.dtype)
    x = x.contiguous()
    f = f.contiguous() if (hk or hv) else None
    meta.grad_mode = torch.is_grad_enabled()
    return _ETStack.apply(meta, x, f, C.contiguous(), u.contiguous(), r, *params)
