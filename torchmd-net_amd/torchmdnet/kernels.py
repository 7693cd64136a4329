"""Autograd bindings of the HIP hot path (``include/tmdnet.h``).

Every Function below runs its forward AND its first backward as HIP kernels of
``libtmdnet_hip.so``.  The backward is itself a differentiable Function, so forces obtained with
``create_graph=True`` (reference ``models/model.py:286-298``) can be differentiated again for
force-loss training; that second-order step is expressed with composite PyTorch ops on the GPU
(recompute + autograd), see DESIGN.md "Double backward".
"""
import ctypes
import math
import os
import weakref

import torch
import torch.nn.functional as F
from torch.autograd import Function

from . import _native as nat

# second orders written out by hand ("hand", default) or autograd over the composites ("composite":
# the reference's double differentiation, kept for A/B checks)
HEAD_SECOND_ORDER = os.environ.get("TMDNET_HEAD_SECOND_ORDER", "hand")
# the head's HVP hands its weight-gradient factor rows to the forward node's backward (A/B switch)
HEAD_HANDOFF = os.environ.get("TMDNET_HEAD_HANDOFF", "1") == "1"
_HEAD_HANDED = []  # weakrefs of head links holding handed-off factor rows (check: head_pending_left)


class _HeadLink:
    """Ties a head's forward node to its force-pass node (the HVP).  In a force-matching loss backward both
    compute weight gradients of the same 12 tensors: whichever runs first leaves its factor rows here
    (``pending`` = (side, (rows, factors))) and returns none; the second runs ONE grouped GEMM over both
    row sets (no engine-side sums of two gradients)."""
    __slots__ = ("fwd", "hvp", "pending", "__weakref__")

    def __init__(self, fwd, hvp):
        self.fwd, self.hvp, self.pending = fwd, hvp, None

    def other_will_run(self, side):
        node = (self.hvp if side == "fwd" else self.fwd)()
        return node is not None and _will_run(node)

    def take(self, side):
        """The other side's pending factor rows (and clear them), or None."""
        p = self.pending
        if p is None or p[0] == side:
            return None
        self.pending = None
        return p[1]

    def leave(self, side, factors):
        self.pending = (side, factors)
        _HEAD_HANDED[:] = [r for r in _HEAD_HANDED if (m := r()) is not None and m.pending is not None]
        _HEAD_HANDED.append(weakref.ref(self))


def head_pending_left():
    """Number of head links whose handed-off factor rows were never consumed (and drop them)."""
    left = [m for m in (r() for r in _HEAD_HANDED) if m is not None and m.pending is not None]
    _HEAD_HANDED.clear()
    for m in left:
        m.pending = None
    return len(left)


# Optional live kernel timing (bench.py): when a list is installed here, the ET message forward
# launches are bracketed by HIP events recorded on the launching stream.
EVENT_PROBE = None


# ----------------------------------------------------------------------------- neighbour graph
class EdgeGraph:
    """Destination-grouped CSR edge list built by ``tmdnet_nl_build``.

    ``src``/``dst`` play the roles of the reference ``edge_index[0]``/``edge_index[1]``; row ``t`` of
    the CSR (``row_ptr[t]:row_ptr[t+1]``) holds every edge whose destination is ``t``.  ``deltas``
    (``pos[src]-pos[dst]``, minimum image) and ``distances`` carry autograd to the positions.
    ``transpose[e]`` is the index of the reversed edge (symmetric lists only).
    """

    def __init__(self, n_nodes, row_ptr, src, dst, transpose, deltas, distances, num_pairs,
                 symmetric, static=False):
        self.n_nodes = n_nodes
        self.row_ptr = row_ptr
        self.src = src
        self.dst = dst
        self.transpose = transpose
        self.deltas = deltas
        self.distances = distances
        self.num_pairs = num_pairs
        self.symmetric = symmetric
        self.cutoff = None  # per-edge CosineCutoff, filled by the model (same for every layer)
        self._edge_index = None
        # static (HIP-graph) mode: per-edge tensors are sized to the capacity, slots beyond the found
        # pairs are inert padding (no CSR row references them) and every per-edge gradient buffer is
        # zero-filled so padding rows contribute nothing to the weight-gradient GEMMs.
        self.static = static
        self.num_pairs_dev = None

    def alloc_edge_grad(self, shape, dtype, device):
        return (torch.zeros if self.static else torch.empty)(shape, dtype=dtype, device=device)

    @property
    def n_edges(self):
        return self.src.shape[0]

    @property
    def edge_index(self):
        if self._edge_index is None:
            self._edge_index = torch.stack([self.src, self.dst]).to(torch.long)
        return self._edge_index

    @staticmethod
    def from_edge_index(edge_index, n_nodes):
        """CSR view of an arbitrary (2, E) edge list.  Returns (graph, perm) with
        ``graph`` edges = ``edge_index[:, perm]``; per-edge tensors must be permuted the same way."""
        dev = edge_index.device
        src = edge_index[0].to(torch.int64)
        dst = edge_index[1].to(torch.int64)
        key = dst * (n_nodes + 1) + src
        perm = torch.argsort(key, stable=True)
        src_s, dst_s = src[perm], dst[perm]
        counts = torch.bincount(dst_s, minlength=n_nodes)
        row_ptr = torch.zeros(n_nodes + 1, dtype=torch.int64, device=dev)
        row_ptr[1:] = torch.cumsum(counts, 0)
        # transpose: position of (dst, src) in the sorted key list
        skey = key[perm]
        rkey = src_s * (n_nodes + 1) + dst_s
        pos = torch.searchsorted(skey, rkey).clamp(max=max(skey.numel() - 1, 0))
        found = skey[pos] == rkey if skey.numel() else torch.zeros(0, dtype=torch.bool, device=dev)
        tr = torch.where(found, pos, torch.full_like(pos, -1))
        g = EdgeGraph(n_nodes, row_ptr.to(torch.int32), src_s.to(torch.int32), dst_s.to(torch.int32),
                      tr.to(torch.int32), None, None, int(src.numel()),
                      bool(found.all().item()) if found.numel() else True)
        return g, perm


def _box9(box):
    if box is None or box.numel() == 0:
        return None
    vals = [float(v) for v in box.detach().cpu().reshape(-1).tolist()]
    return (ctypes.c_double * 9)(*vals)


_STRATEGY = {"brute": nat.NL_BRUTE, "shared": nat.NL_SHARED, "cell": nat.NL_CELL}


def neighbor_pairs_raw(strategy, pos, batch, box, use_periodic, cutoff_lower, cutoff_upper,
                       max_pairs, loop, include_transpose, pad_output=True, want_csr=False, pairs_out=None):
    """Launch ``tmdnet_nl_build``.  Returns (neighbors, deltas, distances, num_pairs, row_ptr, T).
    ``pairs_out`` = (pair_row [max_pairs], pair_edge [slots]) int32: also number the edge pairs in the
    same launches (``tmdnet_nl_build_paired``; sorted-row strategies with the transpose map)."""
    lib = nat.load()
    nat.require_gpu(pos, "get_neighbor_pairs")
    if strategy not in _STRATEGY:
        raise RuntimeError("Unknown kernel name")
    if pos.dim() != 2 or pos.shape[1] != 3:
        raise RuntimeError('Expected "positions" to have two dimensions with size 3')
    if pos.shape[0] == 0:
        raise RuntimeError('Expected the 1nd dimension size of "positions" to be more than 0')
    if not pos.is_contiguous():
        raise RuntimeError('Expected "positions" to be contiguous')
    if batch.dim() != 1 or batch.shape[0] != pos.shape[0] or batch.dtype != torch.int64 \
            or not batch.is_contiguous():
        raise RuntimeError('Expected "batch" to be a contiguous int64 vector matching "positions"')
    if int(max_pairs) <= 0:
        raise RuntimeError('Expected "max_num_neighbors" to be positive')
    if not float(cutoff_upper) > 0:
        raise RuntimeError('Expected "cutoff" to be positive')
    n = pos.shape[0]
    cap = int(max_pairs)
    dev = pos.device
    st = _STRATEGY[strategy]
    box9 = _box9(box) if (use_periodic or st == nat.NL_CELL) else None
    if st == nat.NL_CELL:
        if box9 is None:
            raise RuntimeError('Expected "box_size" to have shape (3, 3)')
        b = list(box9)
        if any(b[i] != 0 for i in (1, 2, 3, 5, 6, 7)):
            raise RuntimeError('Expected "box_size" to be diagonal')
    ws_bytes = lib.tmdnet_nl_workspace_bytes(n, st, box9, float(cutoff_upper))
    ws = torch.empty(max(int(ws_bytes), 16), dtype=torch.uint8, device=dev)
    nb = torch.empty((2, cap), dtype=torch.int32, device=dev)
    dl = torch.empty((cap, 3), dtype=pos.dtype, device=dev)
    dist = torch.empty((cap,), dtype=pos.dtype, device=dev)
    num = torch.empty((1,), dtype=torch.int32, device=dev)
    row_ptr = torch.empty((n + 1,), dtype=torch.int32, device=dev) if want_csr else None
    tr = torch.empty((cap,), dtype=torch.int32, device=dev) if (want_csr and include_transpose) else None
    args = (nat.dtype_code(pos.dtype), st, nat.ptr(pos), nat.ptr(batch), n, box9, int(bool(use_periodic)),
            float(cutoff_lower), float(cutoff_upper), cap, int(bool(loop)), int(bool(include_transpose)),
            nat.ptr(nb), nat.ptr(dl), nat.ptr(dist), nat.ptr(num), nat.ptr(row_ptr), nat.ptr(tr),
            int(bool(pad_output)), nat.ptr(ws), int(ws.numel()))
    if pairs_out is not None:
        pr, pe = pairs_out
        if tr is None or st == nat.NL_CELL or pr.shape[0] != cap:
            raise RuntimeError("pair numbering in the build needs sorted rows and the transpose map")
        rc = lib.tmdnet_nl_build_paired(*args, nat.ptr(pr), nat.ptr(pe), pe.shape[0], nat.stream(dev))
        nat.check(rc, "tmdnet_nl_build_paired")
    else:
        rc = lib.tmdnet_nl_build(*args, nat.stream(dev))
        nat.check(rc, "tmdnet_nl_build")
    return nb, dl, dist, num, row_ptr, tr


def validate_box(box, cutoff_upper):
    """Reference box checks (neighbors_cpu.cpp:35-56)."""
    if box.dim() != 2 or box.shape != (3, 3):
        raise RuntimeError('Expected "box_vectors" to have shape (3, 3)')
    v = box.detach().cpu().double().tolist()
    c = float(cutoff_upper)
    checks = [(v[0][1] == 0, "box_vectors[0][1] != 0"), (v[0][2] == 0, "box_vectors[0][2] != 0"),
              (v[1][2] == 0, "box_vectors[1][2] != 0"), (v[0][0] >= 2 * c, "box_vectors[0][0] < 2*cutoff"),
              (v[1][1] >= 2 * c, "box_vectors[1][1] < 2*cutoff"), (v[2][2] >= 2 * c, "box_vectors[2][2] < 2*cutoff"),
              (v[0][0] >= 2 * v[1][0], "box_vectors[0][0] < 2*box_vectors[1][0]"),
              (v[0][0] >= 2 * v[2][0], "box_vectors[0][0] < 2*box_vectors[1][0]"),
              (v[1][1] >= 2 * v[2][1], "box_vectors[1][1] < 2*box_vectors[2][1]")]
    for ok, msg in checks:
        if not ok:
            raise RuntimeError("Invalid box vectors: " + msg)


class _NeighborGeom(Function):
    """(pos) -> (deltas, distances, distances alias) of a prebuilt graph; backward = tmdnet_nl_backward.
    The alias is the distances for a second consumer (the ET stack's force pass reads r besides the edge
    geometry): its gradient is summed by the backward kernel, not by an autograd add launch."""

    @staticmethod
    def forward(ctx, pos, graph, deltas, distances):
        ctx.graph = graph
        ctx.set_materialize_grads(False)  # an unused alias stays None (no zero fill + add)
        ctx.save_for_backward(pos, deltas, distances)
        return deltas, distances, distances.view_as(distances)

    @staticmethod
    def backward(ctx, g_deltas, g_dist, g_dist2):
        pos, deltas, distances = ctx.saved_tensors
        if g_dist is None and g_dist2 is not None:
            g_dist, g_dist2 = g_dist2, None
        if g_deltas is None and g_dist is None:
            return None, None, None, None
        gpos = _NeighborGeomBwd.apply(pos, g_deltas, g_dist, deltas, distances, ctx.graph, g_dist2)
        return gpos, None, None, None


class _NeighborGeomBwd(Function):
    @staticmethod
    def forward(ctx, pos, g_deltas, g_dist, deltas, distances, graph, g_dist2=None):
        lib = nat.load()
        n = pos.shape[0]
        gpos = torch.empty_like(pos)
        gd = None if g_deltas is None else g_deltas.contiguous()
        gr = None if g_dist is None else g_dist.contiguous()
        gr2 = None if g_dist2 is None else g_dist2.contiguous()
        rc = lib.tmdnet_nl_backward_multi(nat.dtype_code(pos.dtype), n, nat.ptr(graph.row_ptr),
                                          nat.ptr(graph.transpose), graph.n_edges, nat.ptr(gd), nat.ptr(gr),
                                          nat.ptr(gr2), nat.ptr(deltas), nat.ptr(distances), nat.ptr(gpos),
                                          nat.stream(pos.device))
        nat.check(rc, "tmdnet_nl_backward_multi")
        ctx.graph = graph
        ctx.two = gr2 is not None
        # the second order sees the summed distance gradient (both slots get its gradient); summed there,
        # so a first-order-only pass (inference forces) launches no add
        ctx.save_for_backward(pos, gd, gr, gr2, deltas, distances)
        return gpos

    @staticmethod
    def backward(ctx, ggpos):
        pos, gd, gr, gr2, deltas, distances = ctx.saved_tensors
        gr = _sum_opt([gr, gr2])
        d_pos, d_gd, d_gr = _NeighborGeomBwd2.apply(pos, ggpos, gd, gr, deltas, distances, ctx.graph)
        d_gr = d_gr if gr is not None else None
        return d_pos, (d_gd if gd is not None else None), d_gr, None, None, None, (d_gr if ctx.two else None)


def nl_backward_composite(pos, gd, gr, deltas, distances, src, dst):
    """Differentiable restatement of tmdnet_nl_backward (reference neighbors_cuda.cu:43-71):
    g = gd + delta/r*gr (0 where r == 0); dpos = index_add(src, g) - index_add(dst, g)."""
    # padding slots (-1) have r == 0 and are masked; the upper clamp keeps any out-of-range slot
    # (there is none by the build's contract, tests/test_gpu_capture.py) from becoming a fault
    n = pos.shape[0]
    s, d = src.long().clamp(0, n - 1), dst.long().clamp(0, n - 1)
    shift = (deltas - (pos.index_select(0, s) - pos.index_select(0, d))).detach()
    dl = pos.index_select(0, s) - pos.index_select(0, d) + shift
    zero = distances == 0
    r = torch.where(zero, torch.ones_like(distances), (dl * dl).sum(1)).sqrt()  # no 0/0 through sqrt(0)
    g = torch.zeros_like(dl) if gd is None else gd
    if gr is not None:
        g = g + dl / r.unsqueeze(1) * gr.unsqueeze(1)
    g = torch.where(zero.unsqueeze(1), torch.zeros_like(dl), g)
    return torch.zeros_like(pos).index_add(0, s, g).index_add(0, d, -g)


def nl_backward2_composite(pos, ggpos, gr, deltas, distances, src, dst):
    """Differentiable restatement of tmdnet_nl_backward2: (d_pos, d_gd, d_gr) = the gradient of
    <ggpos, nl_backward_composite(pos, gd, gr, ...)> w.r.t. (pos, gd, gr)."""
    n = pos.shape[0]
    s, d = src.long().clamp(0, n - 1), dst.long().clamp(0, n - 1)
    live = ((distances != 0) & (src >= 0) & (src < n) & (dst >= 0) & (dst < n)).to(pos.dtype).unsqueeze(1)
    shift = (deltas - (pos.index_select(0, s) - pos.index_select(0, d))).detach()
    dl = pos.index_select(0, s) - pos.index_select(0, d) + shift
    r = torch.where(distances == 0, torch.ones_like(distances), (dl * dl).sum(1)).sqrt()
    u = dl / r.unsqueeze(1)
    w = (ggpos.index_select(0, s) - ggpos.index_select(0, d)) * live
    uw = (u * w).sum(1, keepdim=True)
    d_pos = torch.zeros_like(pos)
    if gr is not None:
        h = (gr / r).unsqueeze(1) * (w - u * uw)
        d_pos = d_pos.index_add(0, s, h).index_add(0, d, -h)
    return d_pos, w, uw.squeeze(1)


class _NeighborGeomBwd2(Function):
    """Second order of the neighbour op (HIP tmdnet_nl_backward2); its own backward (third order)
    differentiates the composite."""

    @staticmethod
    def forward(ctx, pos, ggpos, gd, gr, deltas, distances, graph):
        lib = nat.load()
        n = pos.shape[0]
        cap = graph.n_edges
        d_pos = torch.empty_like(pos)
        d_gd = torch.empty((cap, 3), dtype=pos.dtype, device=pos.device) if gd is not None else None
        d_gr = torch.empty((cap,), dtype=pos.dtype, device=pos.device) if gr is not None else None
        gg = ggpos.contiguous()
        rc = lib.tmdnet_nl_backward2(nat.dtype_code(pos.dtype), n, nat.ptr(graph.row_ptr), nat.ptr(graph.src),
                                     nat.ptr(graph.transpose), cap, nat.ptr(gr), nat.ptr(deltas),
                                     nat.ptr(distances), nat.ptr(gg), nat.ptr(d_pos), nat.ptr(d_gd),
                                     nat.ptr(d_gr), nat.stream(pos.device))
        nat.check(rc, "tmdnet_nl_backward2")
        ctx.graph = graph
        ctx.has = (gd is not None, gr is not None)
        ctx.save_for_backward(pos, gg, gr, deltas, distances)
        return d_pos, d_gd, d_gr

    @staticmethod
    def backward(ctx, g_dpos, g_dgd, g_dgr):
        pos, gg, gr, deltas, distances = ctx.saved_tensors
        graph = ctx.graph
        with torch.enable_grad():
            p = pos.detach().requires_grad_(True)
            g_ = gg.detach().requires_grad_(True)
            r_ = None if gr is None else gr.detach().requires_grad_(True)
            outs = nl_backward2_composite(p, g_, r_, deltas, distances, graph.src, graph.dst)
            pairs = [(o, go) for o, go in zip(outs, (g_dpos, g_dgd, g_dgr)) if go is not None]
            ins = (p, g_) + ((r_,) if r_ is not None else ())
            grads = torch.autograd.grad([o for o, _ in pairs], ins, [go for _, go in pairs],
                                        create_graph=True, allow_unused=True)
        d_gr = grads[2] if r_ is not None else None
        return grads[0], grads[1], None, d_gr, None, None, None


class DeviceOverflow:
    """Capacity-overflow status of a static-capacity build, read on demand (``.item()`` syncs) from
    the device pair count -- no comparison kernel inside a captured step."""

    def __init__(self, num_pairs_dev, capacity):
        self.num = num_pairs_dev
        self.capacity = int(capacity)

    def item(self):
        return int(self.num.item()) > self.capacity


def build_graph(pos, batch, cutoff_lower, cutoff_upper, max_num_pairs, loop=True, strategy="brute",
                box=None, check_errors=True, static_capacity=None, pairs=False):
    """Symmetric (include_transpose) neighbour graph with CSR rows, transpose map and autograd
    deltas/distances.  Mirrors OptimizedDistance(return_vecs=True, resize_to_fit=True) semantics
    (reference models/utils.py:207-269): one host sync reads num_pairs for the overflow check.
    With ``static_capacity`` the graph is sync-free and HIP-graph capturable: every per-edge tensor
    has ``static_capacity`` rows; overflow is reported on the device (``graph.overflow``).
    ``pairs``: the pair numbering of ``pair_index`` is produced by the build itself (sorted-row
    strategies; the cell list numbers them lazily with tmdnet_pair_index)."""
    use_periodic = box is not None and box.numel() > 0
    if use_periodic:
        validate_box(box, cutoff_upper)
    if strategy == "cell" and not use_periodic:
        lbox = float(cutoff_upper) * 3.0
        box = torch.tensor([[lbox, 0, 0], [0, lbox, 0], [0, 0, lbox]], dtype=torch.float64)
    if strategy == "brute" and pos.shape[0] >= 32768:
        strategy = "shared"
    n = pos.shape[0]
    fused_pairs = None
    if pairs and strategy != "cell":
        c = int(static_capacity) if static_capacity is not None else int(max_num_pairs)
        fused_pairs = (torch.empty((c,), dtype=torch.int32, device=pos.device),
                       torch.empty(((c + n) // 2,), dtype=torch.int32, device=pos.device))
    if static_capacity is not None:
        cap = int(static_capacity)
        nb, dl, dist, num, row_ptr, tr = neighbor_pairs_raw(
            strategy, pos, batch, box, use_periodic, cutoff_lower, cutoff_upper, cap, loop,
            True, pad_output=True, want_csr=True, pairs_out=fused_pairs)
        graph = EdgeGraph(pos.shape[0], row_ptr, nb[0], nb[1], tr, None, None, None, symmetric=True,
                          static=True)
        graph.num_pairs_dev = num
        graph.overflow = DeviceOverflow(num, cap)
        graph.sorted_rows = strategy != "cell"  # brute / shared rows list sources ascending
        if fused_pairs is not None:
            graph._pairs = fused_pairs
        deltas, distances, distances2 = _NeighborGeom.apply(pos, graph, dl, dist)
        graph.deltas = deltas
        graph.distances = distances
        graph.distances_alias = distances2  # for a second consumer of r (no autograd add of the two)
        return graph
    nb, dl, dist, num, row_ptr, tr = neighbor_pairs_raw(
        strategy, pos, batch, box, use_periodic, cutoff_lower, cutoff_upper, max_num_pairs, loop,
        True, pad_output=False, want_csr=True, pairs_out=fused_pairs)
    num_pairs = int(num.item())
    cap = int(max_num_pairs)
    if check_errors and num_pairs > cap:
        raise RuntimeError("Found num_pairs({}) > max_num_pairs({})".format(num_pairs, cap))
    E = min(num_pairs, cap)
    graph = EdgeGraph(pos.shape[0], row_ptr, nb[0, :E], nb[1, :E], tr[:E], None, None, num_pairs,
                      symmetric=num_pairs <= cap)
    graph.sorted_rows = strategy != "cell"  # brute / shared rows list sources ascending
    if fused_pairs is not None and graph.symmetric:  # the numbering of the kept prefix of rows
        graph._pairs = (fused_pairs[0][:E], fused_pairs[1][:(E + n) // 2])
    deltas, distances, distances2 = _NeighborGeom.apply(pos, graph, dl[:E], dist[:E])
    graph.deltas = deltas
    graph.distances = distances
    graph.distances_alias = distances2
    return graph


# ----------------------------------------------------------------------------- edge geometry
def _cosine_cutoff_torch(r, cl, cu):
    if cl > 0:
        c = 0.5 * (torch.cos(math.pi * (2 * (r - cl) / (cu - cl) + 1.0)) + 1.0)
        return c * (r < cu) * (r > cl)
    return 0.5 * (torch.cos(r * math.pi / cu) + 1.0) * (r < cu)


def _edge_geom_composite(deltas, dist, selfmask, mu, beta, cl, cu, rbf_type, want):
    outs = []
    if want[0]:
        r = dist.unsqueeze(-1)
        if rbf_type == nat.RBF_EXPNORM:
            alpha = 5.0 / (cu - cl)
            f = _cosine_cutoff_torch(r, 0.0, cu) * torch.exp(-beta * (torch.exp(alpha * (-r + cl)) - mu) ** 2)
        else:
            f = torch.exp(beta[0] * (r - mu) ** 2)
        outs.append(f)
    else:
        outs.append(None)
    outs.append(_cosine_cutoff_torch(dist, cl, cu) if want[1] else None)
    if want[2]:
        sq = (deltas * deltas).sum(1)
        n = torch.where(selfmask, torch.ones_like(sq), sq).sqrt().unsqueeze(1)
        outs.append(torch.where(selfmask.unsqueeze(1), deltas, deltas / n))
    else:
        outs.append(None)
    return outs


class _EdgeGeom(Function):
    """(rbf, cutoff, unit vectors) of the graph's edges.  ``fan`` = (k_f, k_c): k_f - 1 more aliases of the
    rbf output and k_c - 1 of the cutoff, one per further consumer; their gradients are summed by the
    backward kernel (tmdnet_edge_geom_bwd_multi) instead of by autograd add launches."""

    @staticmethod
    def forward(ctx, deltas, dist, graph, mu, beta, cl, cu, rbf_type, want, rows_out=None, fan=(1, 1)):
        lib = nat.load()
        E = dist.shape[0]
        R = mu.shape[0]
        f = torch.empty((E, R), dtype=dist.dtype, device=dist.device) if want[0] else None
        C = torch.empty((E,), dtype=dist.dtype, device=dist.device) if want[1] else None
        u = torch.empty((E, 3), dtype=dist.dtype, device=dist.device) if want[2] else None
        args = (nat.dtype_code(dist.dtype), E, R, rbf_type, nat.ptr(graph.src), nat.ptr(graph.dst), nat.ptr(deltas),
                nat.ptr(dist), nat.ptr(mu), nat.ptr(beta), float(cl), float(cu), nat.ptr(f), nat.ptr(C), nat.ptr(u))
        if rows_out is not None:  # also f (and df/dr) at rows (written in place, no autograd: forward-only)
            rows, frows, drows = rows_out
            if drows is not None:
                rc = lib.tmdnet_edge_geom_fwd_rows2(*args, nat.ptr(rows), rows.shape[0], nat.ptr(frows),
                                                    nat.ptr(drows), nat.stream(dist.device))
            else:
                rc = lib.tmdnet_edge_geom_fwd_rows(*args, nat.ptr(rows), rows.shape[0], nat.ptr(frows),
                                                   nat.stream(dist.device))
        else:
            rc = lib.tmdnet_edge_geom_fwd(*args, nat.stream(dist.device))
        nat.check(rc, "tmdnet_edge_geom_fwd")
        ctx.graph = graph
        ctx.cfg = (cl, cu, rbf_type, want)
        ctx.fan = fan
        ctx.set_materialize_grads(False)  # an alias whose consumer sends no gradient stays None (no zero fill)
        ctx.save_for_backward(deltas, dist, mu, beta)
        extra = [f.view_as(f) for _ in range(fan[0] - 1)] + [C.view_as(C) for _ in range(fan[1] - 1)]
        return (f, C, u, *extra)

    @staticmethod
    def backward(ctx, gf, gC, gu, *galias):
        deltas, dist, mu, beta = ctx.saved_tensors
        cl, cu, rbf_type, want = ctx.cfg
        kf = ctx.fan[0] - 1
        gfs = [gf] + list(galias[:kf])
        gCs = [gC] + list(galias[kf:])
        gfs += [None] * (3 - len(gfs))
        gCs += [None] * (3 - len(gCs))
        if all(t is None for t in gfs + gCs) and gu is None:
            return (None,) * 11
        g_dl, g_r = _EdgeGeomBwd.apply(deltas, dist, gfs[0], gCs[0], gu, ctx.graph, mu, beta, cl, cu, rbf_type,
                                       gfs[1], gfs[2], gCs[1], gCs[2])
        return g_dl, g_r, None, None, None, None, None, None, None, None, None


def _sum_opt(ts):
    live = [t for t in ts if t is not None]
    if not live:
        return None
    out = live[0]
    for t in live[1:]:
        out = out + t
    return out


def _slot_grads(ctx, d_gf, d_gC):
    """Gradients of _EdgeGeomBwd's extra gradient slots (gf2, gf3, gC2, gC3): the same as slot 1's."""
    fs, cs = ctx.slots
    return (d_gf if fs[1] else None, d_gf if fs[2] else None, d_gC if cs[1] else None, d_gC if cs[2] else None)


class _EdgeGeomBwd(Function):
    @staticmethod
    def forward(ctx, deltas, dist, gf, gC, gu, graph, mu, beta, cl, cu, rbf_type, gf2=None, gf3=None, gC2=None,
                gC3=None):
        lib = nat.load()
        E = dist.shape[0]
        R = mu.shape[0]
        g_r = torch.empty_like(dist)
        g_dl = torch.empty_like(deltas)
        c = lambda t: None if t is None else t.contiguous()  # noqa: E731
        gfl = [c(gf), c(gf2), c(gf3)]
        gCl = [c(gC), c(gC2), c(gC3)]
        gu_ = c(gu)
        rc = lib.tmdnet_edge_geom_bwd_multi(nat.dtype_code(dist.dtype), E, R, rbf_type, nat.ptr(graph.src),
                                            nat.ptr(graph.dst), nat.ptr(deltas), nat.ptr(dist), nat.ptr(mu),
                                            nat.ptr(beta), float(cl), float(cu), *[nat.ptr(t) for t in gfl],
                                            *[nat.ptr(t) for t in gCl], nat.ptr(gu_), nat.ptr(g_r), nat.ptr(g_dl),
                                            nat.stream(dist.device))
        nat.check(rc, "tmdnet_edge_geom_bwd_multi")
        ctx.graph = graph
        ctx.cfg = (cl, cu, rbf_type)
        # the second order sees the summed incoming gradients (each slot's gradient is the same)
        ctx.slots = ([t is not None for t in gfl], [t is not None for t in gCl])
        # (summed in backward: a first-order-only pass launches no adds)
        ctx.save_for_backward(deltas, dist, gu_, mu, beta, *gfl, *gCl)
        return g_dl, g_r

    @staticmethod
    def backward(ctx, gg_dl, gg_r):
        deltas, dist, gu, mu, beta, *gs = ctx.saved_tensors
        gf, gC = _sum_opt(gs[:3]), _sum_opt(gs[3:])
        cl, cu, rbf_type = ctx.cfg
        graph = ctx.graph
        _create = torch.is_grad_enabled()  # third order only if the caller builds a graph
        if not _create and HEAD_SECOND_ORDER != "composite":
            # tmdnet_edge_geom_bwd2: only the gradients the engine will consume (a training step's
            # loss.backward(inputs=params) never reaches the positions: no d_dist / d_deltas)
            fs, cs = ctx.slots  # every gradient slot (fan-out) takes the summed slots' gradient
            nf = iter(ctx.next_functions)
            want = []
            for i, present in enumerate((True, True, fs[0], cs[0], gu is not None)):
                node = next(nf)[0] if present else None
                want.append(present and ctx.needs_input_grad[i] and _will_run(node))
            want[2] = gf is not None and (want[2] or any(fs[1:]))
            want[3] = gC is not None and (want[3] or any(cs[1:]))
            if not any(want):
                return (None,) * 15
            o = [torch.empty_like(t) if w else None for t, w in zip((deltas, dist, gf, gC, gu), want)]
            lib = nat.load()
            rc = lib.tmdnet_edge_geom_bwd2(
                nat.dtype_code(dist.dtype), dist.shape[0], mu.shape[0], rbf_type, nat.ptr(graph.src),
                nat.ptr(graph.dst), nat.ptr(deltas), nat.ptr(dist), nat.ptr(mu), nat.ptr(beta), float(cl), float(cu),
                nat.ptr(gf), nat.ptr(gC), nat.ptr(gu), nat.ptr(None if gg_dl is None else gg_dl.contiguous()),
                nat.ptr(None if gg_r is None else gg_r.contiguous()), nat.ptr(o[2]), nat.ptr(o[3]), nat.ptr(o[4]),
                nat.ptr(o[1]), nat.ptr(o[0]), nat.stream(dist.device))
            nat.check(rc, "tmdnet_edge_geom_bwd2")
            return (o[0], o[1], o[2] if fs[0] else None, o[3] if cs[0] else None, o[4], None, None, None, None, None,
                    None) + _slot_grads(ctx, o[2], o[3])
        selfmask = graph.src == graph.dst
        with torch.enable_grad():
            dl = deltas.detach().requires_grad_(True)
            r = dist.detach().requires_grad_(True)
            ups = [None if t is None else t.detach().requires_grad_(True) for t in (gf, gC, gu)]
            want = tuple(t is not None for t in ups)
            outs = _edge_geom_composite(dl, r, selfmask, mu, beta, cl, cu, rbf_type, want)
            pairs = [(o, g) for o, g in zip(outs, ups) if g is not None]
            first = torch.autograd.grad([o for o, _ in pairs], (dl, r), [g for _, g in pairs],
                                        create_graph=True, allow_unused=True)
            inputs = [dl, r] + [u for u in ups if u is not None]
            sel = [(f, g) for f, g in zip(first, (gg_dl, gg_r)) if f is not None and g is not None]
            if not sel:
                return (None,) * 15
            second = torch.autograd.grad([f for f, _ in sel], inputs, [g for _, g in sel],
                                         create_graph=_create, allow_unused=True)
        it = iter(second[2:])
        gups = [next(it) if u is not None else None for u in ups]
        fs, cs = ctx.slots
        return (second[0], second[1], gups[0] if fs[0] else None, gups[1] if cs[0] else None, gups[2], None, None,
                None, None, None, None) + _slot_grads(ctx, gups[0], gups[1])


def rbf_deriv_launch(r, mu, beta, cl, cu, rbf_type, rows, out):
    lib = nat.load()
    rc = lib.tmdnet_rbf_deriv(nat.dtype_code(r.dtype), mu.shape[0], rbf_type, nat.ptr(r), nat.ptr(mu),
                              nat.ptr(beta), float(cl), float(cu), nat.ptr(rows), out.shape[0], nat.ptr(out),
                              nat.stream(r.device))
    nat.check(rc, "tmdnet_rbf_deriv")


def rbf_deriv(r, mu, beta, cl, cu, rbf_type, rows=None):
    """d f / d r [n, R] of the RBF features (the fused edge-geometry basis) at r[rows] (rows None:
    every edge) -- tmdnet_rbf_deriv."""
    n = r.shape[0] if rows is None else rows.shape[0]
    out = torch.empty((n, mu.shape[0]), dtype=r.dtype, device=r.device)
    if n:
        rbf_deriv_launch(r.detach(), mu.detach(), beta.detach(), cl, cu, rbf_type, rows, out)
    return out


def rbf_composite(r, mu, beta, cl, cu, rbf_type):
    """Differentiable PyTorch RBF features of distances r (same basis as tmdnet_edge_geom_fwd)."""
    return _edge_geom_composite(None, r, None, mu, beta, cl, cu, rbf_type, (True, False, False))[0]


def edge_geometry(graph, mu, beta, cutoff_lower, cutoff_upper, rbf_type, want=(True, True, True), rows=None,
                  fan=(1, 1), drows=False):
    """(rbf [E,R], cutoff [E], unit vectors [E,3]) of the graph's edges, fused (one HIP kernel).
    ``rows`` (int32 [P]): also returns the rbf rows of those edges [P,R] from the same launch (a
    forward-only tensor: gradients flow through the per-edge rbf), as a fourth value -- and with
    ``drows``, their r-derivatives [P,R] as a fifth (the dr-mode force pass's operand).
    ``fan`` = (k_f, k_c), each <= 3: returns ([rbf aliases] * k_f, [cutoff aliases] * k_c, unit) instead --
    one alias per consumer, whose gradients the backward kernel sums (no autograd add launches)."""
    rows_out = None
    if rows is not None:
        mk = lambda: torch.empty((rows.shape[0], mu.shape[0]), dtype=graph.distances.dtype,  # noqa: E731
                                 device=graph.distances.device)
        rows_out = (rows, mk(), mk() if drows else None)
    fan = (max(1, min(3, int(fan[0]))), max(1, min(3, int(fan[1]))))
    if fan != (1, 1) and not (want[0] and want[1]):
        raise ValueError("edge_geometry: fan-out needs the rbf and cutoff outputs")
    out = _EdgeGeom.apply(graph.deltas, graph.distances, graph, mu.detach(), beta.detach(),
                          float(cutoff_lower), float(cutoff_upper), rbf_type, tuple(want), rows_out, fan)
    if fan != (1, 1):
        f, C, u = out[0], out[1], out[2]
        extra = out[3:]
        fs = [f] + list(extra[:fan[0] - 1])
        Cs = [C] + list(extra[fan[0] - 1:])
        res = (fs, Cs, u)
    else:
        res = tuple(out[:3])
    if rows is None:
        return res
    return res + (rows_out[1],) + ((rows_out[2],) if drows else ())


# ----------------------------------------------------------------------------- ET message
def _ld(t):
    return 0 if t is None else t.stride(0)


def rows_like(t, alloc=torch.empty):
    """Gradient buffer with the same row stride as ``t`` (kernels write gradients with the input's
    leading dimension)."""
    if t is None:
        return None
    if t.stride(0) == t.shape[1]:
        return alloc(tuple(t.shape), dtype=t.dtype, device=t.device)
    return alloc((t.shape[0], t.stride(0)), dtype=t.dtype, device=t.device)[:, :t.shape[1]]


def et_message_fwd_launch(q, k, v, vec, pk, pv, C, u, graph, heads, xo, vo, flags=0, pk_rows=None):
    """One ``tmdnet_et_message_fwd`` launch (vec may be None: vec == 0; flags: nat.ET_V_PLANAR;
    pk_rows: edge e reads pk / pv row pk_rows[e], the pair-shared rows of ``pair_index``)."""
    lib = nat.load()
    N, H = q.shape
    probe = EVENT_PROBE
    if probe is not None:
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
    rc = lib.tmdnet_et_message_fwd(nat.dtype_code(q.dtype), N, H, heads, nat.ptr(graph.row_ptr),
                                   nat.ptr(graph.src), graph.n_edges, nat.ptr(q), _ld(q), nat.ptr(k),
                                   _ld(k), nat.ptr(v), _ld(v), nat.ptr(vec), nat.ptr(pk), _ld(pk),
                                   nat.ptr(pv), _ld(pv), nat.ptr(C), nat.ptr(u), nat.ptr(xo),
                                   nat.ptr(vo), int(flags), nat.ptr(pk_rows), None, nat.stream(q.device))
    nat.check(rc, "tmdnet_et_message_fwd")
    if probe is not None:
        ev1.record()
        probe.append((ev0, ev1, graph.n_edges, N, H))


def fep_split(W, b):
    """The fused-projection weight image of one layer (``tmdnet_fep_split_f32``): W [D, R] = the
    layer's [dk | dv] rows in the planar order, b [D].  Returns (img, wsc, bias) device tensors."""
    lib = nat.load()
    D, R = W.shape
    img = torch.empty(int(lib.tmdnet_fep_image_bytes(D, R)) // 2, dtype=torch.float16, device=W.device)
    wsc = torch.empty(D, dtype=torch.float32, device=W.device)
    bo = torch.empty(D, dtype=torch.float32, device=W.device)
    rc = lib.tmdnet_fep_split_f32(D, R, nat.ptr(W), _ld(W), nat.ptr(b), nat.ptr(img), nat.ptr(wsc), nat.ptr(bo),
                                  nat.stream(W.device))
    nat.check(rc, "tmdnet_fep_split_f32")
    return img, wsc, bo


def fep_supported(H, heads, R, dtype):
    """Shapes / dtype the fused dk/dv projection kernels take (tmdnet_et_fused_fwd_f32)."""
    return H == 128 and heads == 8 and R in (32, 64) and dtype == torch.float32


def fep_frags(r_rows, mu, beta, cl, cu, rbf_type):
    """The RBF / d RBF / d r MFMA fragments of the fused kernels for projection rows at distances r_rows
    (``tmdnet_fep_frags_f32``; once per evaluation, every layer reads them).  Returns (frags, dscale)."""
    lib = nat.load()
    rows, R = int(r_rows.shape[0]), int(mu.shape[0])
    fr = torch.empty(max(1, int(lib.tmdnet_fep_frags_bytes(rows, R)) // 2), dtype=torch.float16,
                     device=r_rows.device)
    dsc = torch.empty(max(1, rows), dtype=torch.float32, device=r_rows.device)
    rc = lib.tmdnet_fep_frags_f32(rows, R, nat.ptr(r_rows.contiguous()), nat.ptr(mu.contiguous()),
                                  nat.ptr(beta.contiguous()), float(cl), float(cu), int(rbf_type), nat.ptr(fr),
                                  nat.ptr(dsc), nat.stream(r_rows.device))
    nat.check(rc, "tmdnet_fep_frags_f32")
    return fr, dsc


def fep_frag_set(graph, r, rbf, pairs=None):
    """(frag_rows [E] int32, frags, dscale, rows): the fragment set of one evaluation -- per pair row when
    the graph has pair numbers (both directions of a pair read one row), else per edge."""
    mu, beta, cl, cu, rt = rbf
    if pairs is not None:
        frag_rows, r_rows = pairs[0], r.detach().index_select(0, pairs[1].long())
    else:
        frag_rows = torch.arange(graph.n_edges, dtype=torch.int32, device=r.device)
        r_rows = r.detach()
    fr, dsc = fep_frags(r_rows, mu, beta, cl, cu, rt)
    return frag_rows, fr, dsc, int(r_rows.shape[0])


def fep_frag_shared(graph, r, rbf):
    """fep_frag_set(graph, r, rbf) cached on the graph: the fused neighbour embedding and the fused layer
    stack of one evaluation read the same fragments (keyed on r's storage and the basis)."""
    mu, beta, cl, cu, rt = rbf
    key = (r.data_ptr(), int(r.shape[0]), mu.data_ptr(), beta.data_ptr(), float(cl), float(cu), int(rt))
    cached = getattr(graph, "_fep_frag", None)
    if cached is not None and cached[0] == key:
        return cached[1]
    pairs = pair_index(graph) if (graph.symmetric and graph.transpose is not None) else None
    frag = fep_frag_set(graph, r, rbf, pairs)
    graph._fep_frag = (key, frag)
    return frag


def et_fused_fwd_launch(q, k, v, vec, C, u, fep, frag, graph, heads, xo, vo, flags=0):
    """One ``tmdnet_et_fused_fwd_f32`` launch: the ET message with the dk/dv projection fused in
    (``fep`` = fep_split(W, b) of the layer; ``frag`` = fep_frag_set(...) of the evaluation);
    ``flags``: nat.ET_V_PLANAR when v is in the planar layout."""
    lib = nat.load()
    N, H = q.shape
    img, wsc, bo = fep
    frag_rows, fr, _, rows = frag
    probe = EVENT_PROBE
    if probe is not None:
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
    rc = lib.tmdnet_et_fused_fwd_f32(N, H, heads, img.numel() // (2 * 4 * H), nat.ptr(graph.row_ptr),
                                     nat.ptr(graph.src), graph.n_edges, nat.ptr(q), _ld(q), nat.ptr(k), _ld(k),
                                     nat.ptr(v), _ld(v), nat.ptr(vec), nat.ptr(C), nat.ptr(u), nat.ptr(frag_rows),
                                     nat.ptr(fr), rows, nat.ptr(img), nat.ptr(wsc), nat.ptr(bo), nat.ptr(xo),
                                     nat.ptr(vo), int(flags) & nat.ET_V_PLANAR, nat.stream(q.device))
    nat.check(rc, "tmdnet_et_fused_fwd_f32")
    if probe is not None:
        ev1.record()
        probe.append((ev0, ev1, graph.n_edges, N, H))


def et_fused_bwd_launch(q, k, v, vec, C, u, fep, frag, graph, heads, gx, gvec, gq, gk, gv, gw, gC, gu, g_r,
                        accumulate=0):
    """``tmdnet_et_fused_bwd_f32``: the fused message's force-pass backward (dr mode: g_r accumulated,
    no projection rows); gradients land in the given buffers with their inputs' row strides."""
    if gq.stride(0) != q.stride(0) or gk.stride(0) != k.stride(0) or gv.stride(0) != v.stride(0):
        raise ValueError("et_fused_bwd: gradients must have the row strides of q / k / v")
    lib = nat.load()
    N, H = q.shape
    img, wsc, bo = fep
    frag_rows, fr, dsc, rows = frag
    cap = graph.n_edges
    wsb = int(lib.tmdnet_et_fused_bwd_workspace_bytes(cap))
    ws = torch.empty(max(1, wsb // 4), dtype=torch.float32, device=q.device) if wsb else None
    rc = lib.tmdnet_et_fused_bwd_f32(N, H, heads, img.numel() // (2 * 4 * H), nat.ptr(graph.row_ptr),
                                     nat.ptr(graph.src), cap, nat.ptr(q), _ld(q), nat.ptr(k), _ld(k), nat.ptr(v),
                                     _ld(v), nat.ptr(vec), nat.ptr(C), nat.ptr(u), nat.ptr(frag_rows), nat.ptr(fr),
                                     nat.ptr(dsc), rows, nat.ptr(img), nat.ptr(wsc), nat.ptr(bo), nat.ptr(gx),
                                     nat.ptr(gvec), nat.ptr(gq), nat.ptr(gk), nat.ptr(gv), nat.ptr(gw), nat.ptr(gC),
                                     nat.ptr(gu), nat.ptr(g_r), int(accumulate), nat.ptr(ws), wsb,
                                     nat.stream(q.device))
    nat.check(rc, "tmdnet_et_fused_bwd_f32")


# The message backward's source pass (and the merged dr-mode pass, k_bwd_merged) reads an edge's
# cutoff, unit vector and projection row for its REVERSED edge: valid only for symmetric lists with
# C[rev(e)] == C[e], unit[rev(e)] == -unit[e] and one projection row per pair (include/tmdnet.h,
# tmdnet_et_message_bwd).  The debug library (TMDNET_LIB=debug) or TMDNET_CHECK_SYMMETRY=1 verifies
# that on the device before every launch (a host sync: diagnostics only).
CHECK_SYMMETRY = os.environ.get("TMDNET_LIB") == "debug" or os.environ.get("TMDNET_CHECK_SYMMETRY") == "1"


# run-time size switches of the message backward's launch forms (include/tmdnet.h tmdnet_set_tuning)
TUNE_ET_BOTH_MAX_NODES, TUNE_ET_MERGED_MIN_NODES = 1, 2


def set_tuning(key, value):
    """Set a launch-form size switch of the HIP library; returns the previous value."""
    prev = int(nat.load().tmdnet_set_tuning(int(key), int(value)))
    if prev < 0:
        raise ValueError(f"tmdnet_set_tuning: unknown key {key}")
    return prev


def check_pair_symmetry(graph, C, u, pk_rows=None):
    """Raise unless the per-edge inputs of the message backward are pair-symmetric over the graph's
    valid edges (see CHECK_SYMMETRY)."""
    tr = graph.transpose
    if tr is None:
        raise RuntimeError("et_message_bwd: the source pass needs a symmetric edge list (transpose map)")
    n = int(graph.row_ptr[graph.n_nodes].item())
    t = tr[:n].long()
    if n and bool((t < 0).any()):
        raise RuntimeError("et_message_bwd: edge without a reverse edge (asymmetric list)")
    if not torch.equal(C[:n][t], C[:n]):
        raise RuntimeError("et_message_bwd: cutoff not pair-symmetric (C[rev(e)] != C[e])")
    if not torch.equal(u[:n][t], -u[:n]):
        raise RuntimeError("et_message_bwd: unit vectors not antisymmetric (u[rev(e)] != -u[e])")
    if pk_rows is not None and not torch.equal(pk_rows[:n][t], pk_rows[:n]):
        raise RuntimeError("et_message_bwd: the two edges of a pair read different projection rows")


def et_message_bwd_launch(q, k, v, vec, pk, pv, C, u, graph, heads, gx, gvec, gq, gk, gv, gw, gpk,
                          gpv, gC, gu, accumulate=0, pk_rows=None, dpk=None, dpv=None, g_r=None):
    """dr mode (g_r given): gpk / gpv stay None and <g_pk, dpk> + <g_pv, dpv> accumulates into g_r
    (dpk / dpv are read with pk's / pv's leading dimensions)."""
    if (dpk is not None and pk is not None and dpk.stride(0) != pk.stride(0)) or \
            (dpv is not None and pv is not None and dpv.stride(0) != pv.stride(0)):
        raise ValueError("et_message_bwd: dpk / dpv must have the row stride of pk / pv")
    # the kernels write each gradient with its input's row stride (gq: q's, gk: k's, gv: v's, gpk: pk's)
    for gt, t in ((gq, q), (gk, k), (gv, v), (gpk, pk), (gpv, pv)):
        if gt is not None and t is not None and gt.stride(0) != t.stride(0):
            raise ValueError("et_message_bwd: gradient buffers must have the row strides of their inputs")
    if CHECK_SYMMETRY:
        check_pair_symmetry(graph, C, u, pk_rows)
    lib = nat.load()
    N, H = q.shape
    rc = lib.tmdnet_et_message_bwd(
        nat.dtype_code(q.dtype), N, H, heads, nat.ptr(graph.row_ptr), nat.ptr(graph.src), graph.n_edges,
        nat.ptr(q), _ld(q), nat.ptr(k), _ld(k), nat.ptr(v), _ld(v), nat.ptr(vec), nat.ptr(pk),
        _ld(pk), nat.ptr(pv), _ld(pv), nat.ptr(C), nat.ptr(u), nat.ptr(gx), nat.ptr(gvec),
        nat.ptr(gq), nat.ptr(gk), nat.ptr(gv), nat.ptr(gw), nat.ptr(gpk), nat.ptr(gpv),
        nat.ptr(gC), nat.ptr(gu), nat.ptr(dpk), nat.ptr(dpv), nat.ptr(g_r), int(accumulate),
        nat.ptr(pk_rows), None, nat.stream(q.device))
    nat.check(rc, "tmdnet_et_message_bwd")


def pair_index_launch(graph, pair_row, pair_edge):
    lib = nat.load()
    n = graph.n_nodes
    ws = torch.empty(int(lib.tmdnet_pair_index_workspace_bytes(n)), dtype=torch.uint8, device=pair_row.device)
    rc = lib.tmdnet_pair_index(n, nat.ptr(graph.row_ptr), nat.ptr(graph.src), nat.ptr(graph.dst),
                               nat.ptr(graph.transpose), graph.n_edges, nat.ptr(graph.num_pairs_dev),
                               int(getattr(graph, "sorted_rows", False)), nat.ptr(pair_row),
                               nat.ptr(pair_edge), pair_edge.shape[0], nat.ptr(ws), ws.numel(),
                               nat.stream(pair_row.device))
    nat.check(rc, "tmdnet_pair_index")


def pair_index(graph):
    """(pair_row [E], pair_edge [P]) of a symmetric graph, cached on it: the two directions of a
    pair share one dk/dv projection row (tmdnet_pair_index).  P = (E + N) // 2 slots bound the pair
    count (every pair but the self loops has two edges); unused slots point at edge 0."""
    cached = getattr(graph, "_pairs", None)
    if cached is not None:
        return cached
    dev = graph.src.device
    pair_row = torch.empty(graph.n_edges, dtype=torch.int32, device=dev)
    pair_edge = torch.empty((graph.n_edges + graph.n_nodes) // 2, dtype=torch.int32, device=dev)
    pair_index_launch(graph, pair_row, pair_edge)
    graph._pairs = (pair_row, pair_edge)
    return graph._pairs


def _rowmajor(t):
    """Rows may be strided (e.g. views into a fused projection) but elements must be contiguous."""
    if t is None:
        return None
    if t.stride(-1) != 1:
        t = t.contiguous()
    return t


# ET message activations (include/tmdnet.h TMDNET_ET_ACT): the reference act_class_mapping
# (models/utils.py:579-584) by module class, coded in bits 8-11 (dk / dv) and 12-15 (attention) of the
# message entry points' flags
ACT_CODES = {"SiLU": 0, "ShiftedSoftplus": 1, "Tanh": 2, "Sigmoid": 3}
SSP_SHIFT = 0.693147182464599609375  # log 2 rounded to fp32, as the reference's ShiftedSoftplus.shift
_ACT_FNS = {0: F.silu, 1: lambda x: F.softplus(x) - SSP_SHIFT, 2: torch.tanh, 3: torch.sigmoid}


def act_code(module):
    """The kernels' code of an activation module (SiLU / ShiftedSoftplus / Tanh / Sigmoid)."""
    code = ACT_CODES.get(type(module).__name__)
    if code is None:
        raise NotImplementedError(f"torchmd-net_amd: no ET kernel activation for {type(module).__name__}")
    return code


def et_act_flags(act_kv, act_attn):
    """Flags bits selecting the dk/dv projection activation and the attention activation."""
    return (int(act_kv) << 8) | (int(act_attn) << 12)


def et_act_fns(acts):
    """(dk/dv activation, attention activation) functions of a flags word."""
    return _ACT_FNS[(acts >> 8) & 15], _ACT_FNS[(acts >> 12) & 15]


def et_message_composite(q, k, v, vec, pk, pv, C, u, src, dst, n_nodes, heads, acts=0):
    """PyTorch restatement of torchmd_et.py:314-347 (used for the second-order backward only);
    ``acts``: the activation bits of the kernels' flags (et_act_flags)."""
    act_kv, act_at = et_act_fns(acts)
    H = q.shape[1]
    d = H // heads
    valid = (src >= 0).to(q.dtype)  # static-capacity padding slots (-1) carry no message
    src, dst = src.clamp(min=0), dst.clamp(min=0)
    qi = q.index_select(0, dst).view(-1, heads, d)
    kj = k.index_select(0, src).view(-1, heads, d)
    s = qi * kj
    if pk is not None:
        s = s * act_kv(pk).view(-1, heads, d)
    attn = act_at(s.sum(-1)) * C.unsqueeze(1)
    vj = v.index_select(0, src).view(-1, heads, 3 * d)
    if pv is not None:
        vj = vj * act_kv(pv).view(-1, heads, 3 * d)
    x, v1, v2 = torch.split(vj, d, dim=2)
    xm = x * (attn * valid.unsqueeze(1)).unsqueeze(2)
    vecj = vec.index_select(0, src).view(-1, 3, heads, d)
    vm = (vecj * v1.unsqueeze(1) + v2.unsqueeze(1) * u.view(-1, 3, 1, 1)) * valid.view(-1, 1, 1, 1)
    xo = torch.zeros((n_nodes, heads, d), dtype=q.dtype, device=q.device).index_add(0, dst, xm)
    vo = torch.zeros((n_nodes, 3, heads, d), dtype=q.dtype, device=q.device).index_add(0, dst, vm)
    return xo.view(n_nodes, H), vo.view(n_nodes, 3, H)


class _ETMessage(Function):
    @staticmethod
    def forward(ctx, q, k, v, vec, pk, pv, C, u, graph, heads, acts=0):
        N, H = q.shape
        xo = torch.empty((N, H), dtype=q.dtype, device=q.device)
        vo = torch.empty((N, 3, H), dtype=q.dtype, device=q.device)
        et_message_fwd_launch(q, k, v, vec, pk, pv, C, u, graph, heads, xo, vo, flags=acts)
        ctx.graph = graph
        ctx.heads = heads
        ctx.acts = acts
        ctx.save_for_backward(q, k, v, vec, pk, pv, C, u)
        return xo, vo

    @staticmethod
    def backward(ctx, gx, gvec):
        q, k, v, vec, pk, pv, C, u = ctx.saved_tensors
        if gx is None:
            gx = torch.zeros((q.shape[0], q.shape[1]), dtype=q.dtype, device=q.device)
        if gvec is None:
            gvec = torch.zeros((q.shape[0], 3, q.shape[1]), dtype=q.dtype, device=q.device)
        outs = _ETMessageBwd.apply(gx.contiguous(), gvec.contiguous(), q, k, v, vec, pk, pv, C, u,
                                   ctx.graph, ctx.heads, ctx.acts)
        gq, gk, gv, gw, gpk, gpv, gC, gu = outs
        return gq, gk, gv, gw, (gpk if pk is not None else None), (gpv if pv is not None else None), \
            gC, gu, None, None, None


class _ETMessageBwd(Function):
    @staticmethod
    def forward(ctx, gx, gvec, q, k, v, vec, pk, pv, C, u, graph, heads, acts=0):
        if not graph.symmetric:
            raise RuntimeError("torchmd-net_amd: the ET backward source pass needs a symmetric edge "
                               "list (include_transpose=True, no capacity overflow)")
        N, H = q.shape
        E = graph.n_edges
        o = dict(dtype=q.dtype, device=q.device)
        gq, gk, gv = rows_like(q), rows_like(k), rows_like(v)
        gw = torch.empty((N, 3, H), **o)
        # every row is written (static-capacity padding rows with zeros by the kernel): no memsets
        gpk = rows_like(pk) if pk is not None else None
        gpv = rows_like(pv) if pv is not None else None
        gC = torch.empty((E,), **o)
        gu = torch.empty((E, 3), **o)
        et_message_bwd_launch(q, k, v, vec, pk, pv, C, u, graph, heads, gx, gvec, gq, gk, gv, gw,
                              gpk, gpv, gC, gu, accumulate=acts)
        if gpk is None:
            gpk = torch.zeros(0, **o)
        if gpv is None:
            gpv = torch.zeros(0, **o)
        ctx.graph = graph
        ctx.heads = heads
        ctx.acts = acts
        ctx.save_for_backward(gx, gvec, q, k, v, vec, pk, pv, C, u)
        return gq, gk, gv, gw, gpk, gpv, gC, gu

    @staticmethod
    def backward(ctx, *ggs):
        return et_message_bwd2(ctx, ggs)

    @staticmethod
    def composite_backward(ctx, *ggs):
        """Second order by recompute + autograd over the PyTorch restatement (tests only)."""
        saved = ctx.saved_tensors
        graph = ctx.graph
        src, dst = graph.src.long(), graph.dst.long()
        _create = torch.is_grad_enabled()  # third order only if the caller builds a graph
        with torch.enable_grad():
            leaves = [None if t is None else t.detach().requires_grad_(True) for t in saved]
            gx, gvec, q, k, v, vec, pk, pv, C, u = leaves
            xo, vo = et_message_composite(q, k, v, vec, pk, pv, C, u, src, dst, graph.n_nodes, ctx.heads,
                                          ctx.acts)
            wrt = [t for t in (q, k, v, vec, pk, pv, C, u)]
            live = [t for t in wrt if t is not None]
            first = torch.autograd.grad((xo, vo), live, (gx, gvec), create_graph=True, allow_unused=True)
            it = iter(first)
            first_full = [next(it) if t is not None else None for t in wrt]
            sel = [(f, g) for f, g in zip(first_full, ggs) if f is not None and g is not None and g.numel()]
            ins = [t for t in leaves if t is not None]
            if not sel:
                return (None,) * 13
            second = torch.autograd.grad([f for f, _ in sel], ins, [g for _, g in sel],
                                         create_graph=_create, allow_unused=True)
        it = iter(second)
        res = [next(it) if t is not None else None for t in leaves]
        return tuple(res) + (None, None, None)


# the deterministic source pass of tmdnet_et_message_bwd2_ex stores 7H values per edge: used up to
# this scratch size (beyond it the atomic source terms keep the memory flat)
BWD2_SCRATCH_MAX_BYTES = 2 << 30


def et_message_bwd2_launch(q, k, v, vec, pk, pv, C, u, graph, heads, gx, gvec, ggs, flags=0, out=None,
                           pk_rows=None, gg_pkv_scale=None):
    """One ``tmdnet_et_message_bwd2_ex`` launch: the VJP of tmdnet_et_message_bwd (without the vec
    residual) at primals (q, k, v, vec, pk, pv, C, u) and seeds (gx, gvec), for the cotangents
    ``ggs`` = (gg_q, gg_k, gg_v, gg_vec, gg_pk, gg_pv, gg_C, gg_u) of its outputs (None / empty =
    zero; node cotangents may be column blocks of a wider buffer).  pk / pv are per-edge rows, or with
    ``pk_rows`` the pair-shared rows edge e reads at pk_rows[e] (their cotangents / gradients stay
    per edge).  ``gg_pkv_scale`` [E] (with pk_rows): the edge cotangents gg_pk / gg_pv are PAIR rows,
    edge e's being row pk_rows[e] scaled by gg_pkv_scale[e].  Returns (d_gx, d_gvec, d_q, d_k, d_v, d_vec, d_pk, d_pv, d_C, d_u); d_vec is None
    when vec is None, d_pk / d_pv when pk / pv are.

    ``out`` (optional dict) names caller buffers: "gx" [N, H] receives d_gx, "qkv" [N, 5H] d_q | d_k | d_v, "pkv" [E, D]
    d_pk | d_pv, "C" / "u" are ACCUMULATED into (d_C / d_u returned as those buffers), "gvec" receives
    d_gvec added to its contents ("edge_overwrite": True -- "C" / "u" are overwritten, padding rows
    zeroed, instead).  With the graph's transpose map the source-node terms are summed by
    the deterministic source pass (per-edge scratch), otherwise by atomics into zeroed buffers."""
    lib = nat.load()
    out = out or {}
    N, H = q.shape
    E = graph.n_edges
    o = dict(dtype=q.dtype, device=q.device)

    def dense(g, shape):  # rows may be strided (read through the leading dimension)
        return torch.zeros(shape, **o) if (g is None or g.numel() == 0) else _rowmajor(g)

    ggq, ggk, ggv = dense(ggs[0], (N, H)), dense(ggs[1], (N, H)), dense(ggs[2], (N, 3 * H))
    ggw = dense(ggs[3], (N, 3, H)).contiguous()
    if gg_pkv_scale is not None:  # pair rows, read through pk_rows and scaled per edge
        if pk_rows is None:
            raise ValueError("gg_pkv_scale needs pk_rows")
        ggpk = _rowmajor(ggs[4]) if pk is not None else None
        ggpv = _rowmajor(ggs[5]) if pv is not None else None
    else:
        ggpk = dense(ggs[4], (E, H)) if pk is not None else None
        ggpv = dense(ggs[5], (E, 3 * H)) if pv is not None else None
    ggC, ggu = dense(ggs[6], (E,)).contiguous(), dense(ggs[7], (E, 3)).contiguous()
    scratch = None
    if graph.transpose is not None and E * 7 * H * q.element_size() <= BWD2_SCRATCH_MAX_BYTES:
        scratch = torch.empty((E, 7 * H), **o)
    new_node = torch.empty if scratch is not None else torch.zeros  # atomics need zeroed buffers
    d_gx = out["gx"] if "gx" in out else torch.empty((N, H), **o)
    if "qkv" in out:
        d_qkv = out["qkv"]
        if scratch is None:
            d_qkv[:, H:].zero_()
        d_q, d_k, d_v = d_qkv[:, :H], d_qkv[:, H:2 * H], d_qkv[:, 2 * H:5 * H]
    else:
        d_q, d_k, d_v = torch.empty((N, H), **o), new_node((N, H), **o), new_node((N, 3 * H), **o)
    d_vec = new_node((N, 3, H), **o) if vec is not None else None
    if "gvec" in out:
        d_gvec = out["gvec"]
        flags |= nat.BWD2_ACC_GVEC
    else:
        d_gvec = torch.empty((N, 3, H), **o)
    # per-edge outputs: every row written (padding rows with zeros by the kernel)
    d_pk = d_pv = None
    if "pkv" in out:
        hk_w = H if pk is not None else 0
        d_pk = out["pkv"][:, :H] if pk is not None else None
        d_pv = out["pkv"][:, hk_w:hk_w + 3 * H] if pv is not None else None
    else:
        d_pk = torch.empty((E, H), **o) if pk is not None else None
        d_pv = torch.empty((E, 3 * H), **o) if pv is not None else None
    if "C" in out:
        d_C, d_u = out["C"], out["u"]
        if not out.get("edge_overwrite"):  # (the first launch into a buffer overwrites it: no zero fill)
            flags |= nat.BWD2_ACC_EDGE
    else:
        d_C, d_u = torch.empty((E,), **o), torch.empty((E, 3), **o)
    qc, kc, vc, pkc, pvc = (_rowmajor(t) for t in (q, k, v, pk, pv))  # read in place through ld
    gxc, gvc = gx.contiguous(), gvec.contiguous()
    P = nat.ptr
    rc = lib.tmdnet_et_message_bwd2_ex(
        nat.dtype_code(q.dtype), N, H, heads, P(graph.row_ptr), P(graph.src),
        P(graph.transpose if scratch is not None else None), E,
        P(qc), _ld(qc), P(kc), _ld(kc), P(vc), _ld(vc), P(vec), P(pkc), _ld(pkc), P(pvc), _ld(pvc),
        P(C), P(u), P(gxc), P(gvc), P(ggq), _ld(ggq), P(ggk), _ld(ggk), P(ggv), _ld(ggv), P(ggw),
        P(ggpk), _ld(ggpk), P(ggpv), _ld(ggpv), P(ggC), P(ggu), P(d_gx), P(d_gvec),
        P(d_q), _ld(d_q), P(d_k), _ld(d_k), P(d_v), _ld(d_v), P(d_vec), P(d_pk), _ld(d_pk), P(d_pv), _ld(d_pv),
        P(d_C), P(d_u), P(scratch), P(pk_rows), P(gg_pkv_scale), int(flags), nat.stream(q.device))
    nat.check(rc, "tmdnet_et_message_bwd2_ex")
    return d_gx, d_gvec, d_q, d_k, d_v, d_vec, d_pk, d_pv, d_C, d_u


def et_message_bwd2(ctx, ggs):
    """HIP second-order backward of the ET message (``tmdnet_et_message_bwd2``).  Its own backward
    (third order) is not implemented."""
    gx, gvec, q, k, v, vec, pk, pv, C, u = ctx.saved_tensors
    out = et_message_bwd2_launch(q, k, v, vec, pk, pv, C, u, ctx.graph, ctx.heads, gx, gvec, ggs,
                                 flags=getattr(ctx, "acts", 0))
    return tuple(out) + (None, None, None)


def et_message(q, k, v, vec, pk, pv, C, u, graph, heads, acts=0):
    """The ET message + aggregation (HIP, differentiable twice); ``acts`` = et_act_flags(...)."""
    q, k, v, pk, pv = (_rowmajor(t) for t in (q, k, v, pk, pv))
    return _ETMessage.apply(q, k, v, vec.contiguous(), pk, pv, C.contiguous(), u.contiguous(), graph, heads, acts)


# ----------------------------------------------------------------------------- neighbour embedding
def nbr_embed_composite(x, w, C, src, dst, n_nodes):
    keep = ((src != dst) & (src >= 0)).to(x.dtype).unsqueeze(1)
    src, dst = src.clamp(min=0), dst.clamp(min=0)
    m = x.index_select(0, src) * (w * C.unsqueeze(1)) * keep
    return torch.zeros((n_nodes, x.shape[1]), dtype=x.dtype, device=x.device).index_add(0, dst, m)


class _NbrEmbed(Function):
    """x_nb = nbr_embed(x, w, C); with x_self the output is [x_self | x_nb] ([N, 2H], the combine
    Linear's input, reference utils.py:108) written by the same kernel."""

    @staticmethod
    def forward(ctx, x, w, C, graph, x_self=None):
        lib = nat.load()
        N, H = x.shape
        if x_self is None:
            buf = out = torch.empty((N, H), dtype=x.dtype, device=x.device)
        else:
            buf = torch.empty((N, 2 * H), dtype=x.dtype, device=x.device)
            out = buf[:, H:]
        rc = lib.tmdnet_nbr_embed_fwd(nat.dtype_code(x.dtype), N, H, nat.ptr(graph.row_ptr),
                                      nat.ptr(graph.src), graph.n_edges, nat.ptr(x), _ld(x), nat.ptr(w),
                                      _ld(w), nat.ptr(C), nat.ptr(out), out.stride(0), nat.ptr(x_self),
                                      None if x_self is None else nat.ptr(buf), nat.stream(x.device))
        nat.check(rc, "tmdnet_nbr_embed_fwd")
        ctx.graph = graph
        ctx.has_self = x_self is not None
        ctx.save_for_backward(x, w, C)
        return buf

    @staticmethod
    def backward(ctx, gout):
        x, w, C = ctx.saved_tensors
        H = x.shape[1]
        g_self = None
        if gout.stride(-1) != 1:
            gout = gout.contiguous()
        if ctx.has_self:  # the two halves are read in place (row stride 2H)
            g_self, gout = gout[:, :H], gout[:, H:]
        # the embedding rows' gradient only when something consumes it (never in a force pass)
        want_x = bool(ctx.needs_input_grad[0]) and _will_run(ctx.next_functions[0][0])
        gx, gw, gC = _NbrEmbedBwd.apply(gout, x, w, C, ctx.graph, want_x)
        return gx, gw, gC, None, g_self


class _NbrEmbedBwd(Function):
    @staticmethod
    def forward(ctx, gout, x, w, C, graph, want_x=True):
        if not graph.symmetric:
            raise RuntimeError("torchmd-net_amd: neighbour-embedding backward needs a symmetric edge list")
        lib = nat.load()
        N, H = x.shape
        E = graph.n_edges
        gx = torch.empty_like(x, memory_format=torch.contiguous_format) if want_x else None
        # every slot written by the kernel (padding slots zero): no fill
        zbuf = torch.empty((E * (H + 1),), dtype=x.dtype, device=x.device)
        gw, gC = zbuf[:E * H].view(E, H), zbuf[E * H:]
        rc = lib.tmdnet_nbr_embed_bwd(nat.dtype_code(x.dtype), N, H, nat.ptr(graph.row_ptr),
                                      nat.ptr(graph.src), E, nat.ptr(x), _ld(x), nat.ptr(w), _ld(w),
                                      nat.ptr(C), nat.ptr(gout), gout.stride(0), nat.ptr(gx), nat.ptr(gw),
                                      nat.ptr(gC), nat.stream(x.device))
        nat.check(rc, "tmdnet_nbr_embed_bwd")
        ctx.graph = graph
        ctx.save_for_backward(gout, x, w, C)
        return gx, gw, gC

    @staticmethod
    def backward(ctx, ggx, ggw, ggC):
        gout, x, w, C = ctx.saved_tensors
        graph = ctx.graph
        _create = torch.is_grad_enabled()  # third order only if the caller builds a graph
        if not _create and HEAD_SECOND_ORDER != "composite" and graph.transpose is not None:
            nodes = [e[0] for e in ctx.next_functions]  # one per tensor input: gout, x, w, C
            want = [bool(ctx.needs_input_grad[i]) and _will_run(nodes[i]) for i in range(4)]
            if not any(want):
                return (None,) * 6
            N, H = x.shape
            E = graph.n_edges
            d_go = torch.empty((N, H), dtype=x.dtype, device=x.device) if want[0] else None
            d_x = torch.empty((N, H), dtype=x.dtype, device=x.device) if want[1] else None
            # edge outputs: the static-capacity padding slots stay zero (one zero-filled buffer)
            zb = graph.alloc_edge_grad((E * (H + 1),), x.dtype, x.device) if (want[2] or want[3]) else None
            d_w = zb[:E * H].view(E, H) if want[2] else None
            d_C = zb[E * H:] if want[3] else None
            lib = nat.load()
            rc = lib.tmdnet_nbr_embed_bwd2(
                nat.dtype_code(x.dtype), N, H, nat.ptr(graph.row_ptr), nat.ptr(graph.src), nat.ptr(graph.transpose),
                E, nat.ptr(x), _ld(x), nat.ptr(w), _ld(w), nat.ptr(C), nat.ptr(gout), gout.stride(0),
                nat.ptr(None if ggx is None else ggx.contiguous()), nat.ptr(None if ggw is None else ggw.contiguous()),
                nat.ptr(None if ggC is None else ggC.contiguous()), nat.ptr(d_go), nat.ptr(d_x), nat.ptr(d_w),
                nat.ptr(d_C), nat.stream(x.device))
            nat.check(rc, "tmdnet_nbr_embed_bwd2")
            return d_go, d_x, d_w, d_C, None, None
        src, dst = graph.src.long(), graph.dst.long()
        with torch.enable_grad():
            leaves = [t.detach().requires_grad_(True) for t in (gout, x, w, C)]
            go, x_, w_, C_ = leaves
            out = nbr_embed_composite(x_, w_, C_, src, dst, graph.n_nodes)
            first = torch.autograd.grad(out, (x_, w_, C_), go, create_graph=True)
            sel = [(f, g) for f, g in zip(first, (ggx, ggw, ggC)) if g is not None]
            if not sel:
                return (None,) * 6
            second = torch.autograd.grad([f for f, _ in sel], leaves, [g for _, g in sel],
                                         create_graph=_create, allow_unused=True)
        return tuple(second) + (None, None)


def nbr_fused_supported(graph, H, R, dtype):
    """Shapes the fused neighbour embedding takes (tmdnet_nbr_fused_fwd_f32): fp32, H = 128, R = 32 / 64,
    a symmetric list (its force-pass backward reads the edges of each node's own row only)."""
    return H == 128 and R in (32, 64) and dtype == torch.float32 and graph.symmetric


class _NbrEmbedFused(Function):
    """[x_self | x_nb] of the neighbour embedding (reference utils.py:90-108) with distance_proj FUSED in:
    x_nb[t] = sum_{e in row t, s != t} x[s] (W rbf(r_e) + b) C_e, the projection formed per tile on the MFMA
    (tmdnet_nbr_fused_fwd_f32) -- no E x H rows.  Backward: the force pass (only r / C gradients wanted,
    no graph) runs tmdnet_nbr_fused_bwd_f32 (dr mode: g_r and g_C per edge); anything else (parameter or
    embedding gradients, create_graph) differentiates the composite restatement through ``rbf_fn``."""

    @staticmethod
    def forward(ctx, x, r, C, W, b, graph, rbf, x_self, rbf_fn):
        lib = nat.load()
        N, H = x.shape
        R = W.shape[1]
        frag = fep_frag_shared(graph, r, rbf)
        img = fep_split(W.detach().contiguous(), b.detach().contiguous())
        if x_self is None:
            buf = out = torch.empty((N, H), dtype=x.dtype, device=x.device)
        else:
            buf = torch.empty((N, 2 * H), dtype=x.dtype, device=x.device)
            out = buf[:, H:]
        frag_rows, fr, _, rows = frag
        rc = lib.tmdnet_nbr_fused_fwd_f32(N, H, R, nat.ptr(graph.row_ptr), nat.ptr(graph.src), graph.n_edges,
                                          nat.ptr(x), _ld(x), nat.ptr(C), nat.ptr(frag_rows), nat.ptr(fr), rows,
                                          nat.ptr(img[0]), nat.ptr(img[1]), nat.ptr(img[2]), nat.ptr(out),
                                          out.stride(0), nat.ptr(x_self), None if x_self is None else nat.ptr(buf),
                                          nat.stream(x.device))
        nat.check(rc, "tmdnet_nbr_fused_fwd_f32")
        ctx.graph, ctx.frag, ctx.img, ctx.rbf_fn = graph, frag, img, rbf_fn
        ctx.has_self = x_self is not None
        ctx.save_for_backward(x, r, C, W, b)
        return buf

    @staticmethod
    def backward(ctx, gout):
        x, r, C, W, b = ctx.saved_tensors
        graph = ctx.graph
        N, H = x.shape
        g_self = None
        if gout.stride(-1) != 1:
            gout = gout.contiguous()
        if ctx.has_self:
            g_self, gout = gout[:, :H], gout[:, H:]
        nodes = [e[0] for e in ctx.next_functions]
        want = [bool(ctx.needs_input_grad[i]) and _will_run(nodes[i]) for i in range(5)]
        tail = (None, None, g_self, None)
        if not (want[0] or want[3] or want[4]):  # the force pass: r / C gradients only (dr mode)
            if not (want[1] or want[2]):
                return (None,) * 5 + tail
            g_r, g_C = _NbrEmbedFusedBwd.apply(gout, x, r, C, W, b, graph, ctx.frag, ctx.img, ctx.rbf_fn)
            return (None, g_r if want[1] else None, g_C if want[2] else None, None, None) + tail
        # parameter / embedding gradients: the composite restatement
        with torch.enable_grad():
            leaves = [t.detach().requires_grad_(w) for t, w in zip((x, r, C, W, b), want)]
            out = _nbr_fused_composite(leaves, graph, ctx.rbf_fn)
            req = [t for t, w_ in zip(leaves, want) if w_]
            gs = torch.autograd.grad(out, req, gout, create_graph=torch.is_grad_enabled(), allow_unused=True)
        it = iter(gs)
        return tuple(next(it) if w_ else None for w_ in want) + tail


def _nbr_fused_composite(leaves, graph, rbf_fn):
    """Differentiable restatement of the fused neighbour embedding's x_nb (reference utils.py:90-107)."""
    x, r, C, W, b = leaves
    w = torch.nn.functional.linear(rbf_fn(r), W, b)
    return nbr_embed_composite(x, w, C, graph.src.long(), graph.dst.long(), graph.n_nodes)


class _NbrEmbedFusedBwd(Function):
    """(g_r, g_C) of the fused neighbour embedding in the force pass (tmdnet_nbr_fused_bwd_f32, dr mode);
    differentiable for force-matching training: its backward differentiates the composite restatement
    twice (the second order at large sizes is not a timed configuration)."""

    @staticmethod
    def forward(ctx, gout, x, r, C, W, b, graph, frag, img, rbf_fn):
        lib = nat.load()
        N, H = x.shape
        E = graph.n_edges
        eb = torch.empty((2 * E,), dtype=x.dtype, device=x.device)
        g_C, g_r = eb[:E], eb[E:]
        frag_rows, fr, dsc, rows = frag
        rc = lib.tmdnet_nbr_fused_bwd_f32(N, H, W.shape[1], nat.ptr(graph.row_ptr), nat.ptr(graph.src), E,
                                          nat.ptr(x), _ld(x), nat.ptr(C), nat.ptr(frag_rows), nat.ptr(fr),
                                          nat.ptr(dsc), rows, nat.ptr(img[0]), nat.ptr(img[1]), nat.ptr(img[2]),
                                          nat.ptr(gout), gout.stride(0), nat.ptr(g_C), nat.ptr(g_r), 0,
                                          nat.stream(x.device))
        nat.check(rc, "tmdnet_nbr_fused_bwd_f32")
        ctx.graph, ctx.rbf_fn = graph, rbf_fn
        ctx.save_for_backward(gout, x, r, C, W, b)
        return g_r, g_C

    @staticmethod
    def backward(ctx, gg_r, gg_C):
        saved = ctx.saved_tensors
        sel = [(i, g) for i, g in ((2, gg_r), (3, gg_C)) if g is not None]
        if not sel:
            return (None,) * 10
        with torch.enable_grad():
            leaves = [t.detach().requires_grad_(True) for t in saved]
            out = _nbr_fused_composite(leaves[1:], ctx.graph, ctx.rbf_fn)
            first = torch.autograd.grad(out, [leaves[i] for i, _ in sel], leaves[0], create_graph=True)
            second = torch.autograd.grad(first, leaves, [g for _, g in sel], create_graph=torch.is_grad_enabled(),
                                         allow_unused=True)
        return tuple(g if ctx.needs_input_grad[i] else None for i, g in enumerate(second)) + (None,) * 4


def nbr_embed_fused(x, r, C, W, b, graph, rbf, rbf_fn, x_self=None):
    """The neighbour-embedding aggregation with distance_proj fused (reference utils.py:90-108):
    ``cat([x_self, x_nb], 1)`` (or x_nb) from r directly -- no rbf or projection rows.  ``rbf`` = (mu, beta,
    cutoff_lower, cutoff_upper, rbf_type) of the basis, ``rbf_fn`` its differentiable module (the composite
    backward)."""
    return _NbrEmbedFused.apply(_rowmajor(x), r, C.contiguous(), W, b, graph, rbf,
                                None if x_self is None else x_self.contiguous(), rbf_fn)


def nbr_embed(x, w, C, graph, x_self=None):
    """Neighbour-embedding aggregation (reference utils.py:100-107); ``x_self`` given: returns
    ``cat([x_self, x_nb], 1)`` from the same launch."""
    return _NbrEmbed.apply(_rowmajor(x), _rowmajor(w), C.contiguous(), graph,
                           None if x_self is None else x_self.contiguous())


# ----------------------------------------------------------------------------- activation
def silu_launch(x, scale, out):
    lib = nat.load()
    rows, cols = x.shape
    rc = lib.tmdnet_silu_fwd(nat.dtype_code(x.dtype), rows, cols, nat.ptr(x), x.stride(0), nat.ptr(scale),
                             nat.ptr(out), nat.stream(x.device))
    nat.check(rc, "tmdnet_silu_fwd")


def silu_bwd_launch(x, scale, g, gx, gscale):
    lib = nat.load()
    rows, cols = x.shape
    rc = lib.tmdnet_silu_bwd(nat.dtype_code(x.dtype), rows, cols, nat.ptr(x), x.stride(0), nat.ptr(scale),
                             nat.ptr(g), g.stride(0), nat.ptr(gx), nat.ptr(gscale), nat.stream(x.device))
    nat.check(rc, "tmdnet_silu_bwd")


def _silu_composite(x, scale):
    y = torch.nn.functional.silu(x)
    return y if scale is None else y * scale.unsqueeze(1)


class _Silu(Function):
    @staticmethod
    def forward(ctx, x, scale):
        out = torch.empty(x.shape, dtype=x.dtype, device=x.device)
        silu_launch(x, scale, out)
        ctx.save_for_backward(x, scale)
        return out

    @staticmethod
    def backward(ctx, g):
        x, scale = ctx.saved_tensors
        return _SiluBwd.apply(g.contiguous(), x, scale, ctx.needs_input_grad[1])


class _SiluBwd(Function):
    @staticmethod
    def forward(ctx, g, x, scale, want_scale):
        gx = torch.empty(x.shape, dtype=x.dtype, device=x.device)
        gs = torch.empty(x.shape[0], dtype=x.dtype, device=x.device) if want_scale else None
        silu_bwd_launch(x, scale, g, gx, gs)
        ctx.save_for_backward(g, x, scale)
        return gx, gs

    @staticmethod
    def backward(ctx, ggx, ggs):
        g, x, scale = ctx.saved_tensors
        from .tn_node import _double_backward
        if scale is None:
            d = _double_backward(lambda a: _silu_composite(a, None), [x], [g], [ggx])
            return d[0], d[1], None, None
        d = _double_backward(_silu_composite, [x, scale], [g], [ggx, ggs])
        return d[0], d[1], d[2], None


def fused_act(act, x, scale=None):
    """``act(x) * scale[:, None]`` (scale optional) for a 2-D ``x``; SiLU on a ROCm device runs as one
    HIP pass forward and one backward (``tmdnet_silu_*``), any other activation as the module."""
    if isinstance(act, torch.nn.SiLU) and x.is_cuda and x.dim() == 2 and x.stride(1) == 1:
        return _Silu.apply(x, None if scale is None else scale.contiguous())
    y = act(x)
    return y if scale is None else y * scale.view(-1, 1)


# ----------------------------------------------------------------------------- small grouped GEMM
GEMM_UNSUPPORTED = 2
GEMM_MAX_ROWS = 16384  # the grouped split-K kernel's envelope; above it the x3 GEMM (gemm_x3) takes the rows


def gemm_launch(problems):
    """``tmdnet_gemm_f32``: up to 4 problems (A, B, trans_b, bias, C, beta) in one launch,
    C = beta C + A op(B) + bias.  Returns False (nothing launched) when a problem is outside the
    kernel's envelope (non-fp32, empty, K % 16, alignment); the caller then uses the library GEMM."""
    if any(A.dtype != torch.float32 or not 0 < A.shape[0] <= GEMM_MAX_ROWS or A.shape[1] == 0 or C.shape[1] == 0
           for A, _, _, _, C, _ in problems):
        return False
    lib = nat.load()
    n = len(problems)
    dims = (ctypes.c_int * (8 * n))()
    ptrs = (ctypes.c_void_p * (4 * n))()
    for i, (A, B, tb, bias, C, beta) in enumerate(problems):
        if A.stride(1) != 1 or B.stride(1) != 1 or C.stride(1) != 1:
            return False
        dims[8 * i:8 * i + 8] = [A.shape[0], C.shape[1], A.shape[1], A.stride(0), B.stride(0), C.stride(0),
                                 int(tb), int(beta)]
        ptrs[4 * i:4 * i + 4] = [A.data_ptr(), B.data_ptr(), None if bias is None else bias.data_ptr(),
                                 C.data_ptr()]
    rc = lib.tmdnet_gemm_f32(n, dims, ptrs, nat.stream(problems[0][0].device))
    if rc == GEMM_UNSUPPORTED:
        return False
    nat.check(rc, "tmdnet_gemm_f32")
    return True


# above GEMM_MAX_ROWS (C5-size systems) fp32 GEMMs run on tmdnet_gemm_x3_f32 (bf16 MFMA, exact three-piece
# split, fp32 accuracy); TMDNET_GEMM_BIG=lib keeps the library GEMM there (A/B switch)
GEMM_BIG = os.environ.get("TMDNET_GEMM_BIG", "x3")
# where the weight's bf16 pieces come from: "launch" = a split launch per call (tmdnet_proj_split_f32 /
# tmdnet_split_t_f32, ~5 us each; nothing cached, so in-place weight updates are always seen), "kernel" = split
# inside the GEMM while staged in LDS (tmdnet_gemm_x3w_f32: no split launch, but every workgroup re-splits its
# weight tile -- measured slower: C5 ET 50.8-51.1 vs 48.3-49.1 ms, C5 TensorNet 35.5 vs 34.2 ms per evaluation,
# the transposed form's 2-byte LDS scatter and the split VALU work competing with the MFMA chain)
X3_WSPLIT = os.environ.get("TMDNET_X3_WSPLIT", "launch")


def _al16(*ts):
    return all(t is None or (t.data_ptr() % 16 == 0) for t in ts)


def gemm_x3(A, B, tb, bias, C, beta, act=0, pre=None, rscale=None, dpre=None):
    """``C = beta C + A op(B) + bias`` on ``tmdnet_gemm_x3_f32`` for large row counts: op(B) = B^T for a
    [N][K] Linear weight (split once per call, tmdnet_proj_split_f32), B for a [K][N] right operand
    (tmdnet_split_t_f32).  ``act`` / ``pre`` / ``rscale`` / ``dpre``: tmdnet_gemm_ex_f32's epilogue
    (tmdnet_gemm_x3_ex_f32).  Returns False (nothing launched) outside its envelope (non-fp32, K % 32,
    N % 16, strides / alignment); the caller then uses the library GEMM."""
    M, K = A.shape
    N = C.shape[1]
    x = pre if pre is not None else dpre
    if not (GEMM_BIG == "x3" and A.is_cuda and A.dtype == torch.float32 and B.dtype == torch.float32
            and C.dtype == torch.float32 and M > 0 and K % 32 == 0 and N % 16 == 0 and A.stride(1) == 1
            and B.stride(1) == 1 and C.stride(1) == 1 and A.stride(0) % 4 == 0 and C.stride(0) % 4 == 0
            and B.stride(0) % 4 == 0 and (bias is None or bias.is_contiguous()) and _al16(A, B, C, bias, pre, dpre)
            and (x is None or (x.stride(1) == 1 and x.stride(0) % 4 == 0 and x.shape == C.shape))
            and (pre is None or dpre is None or pre.stride(0) == dpre.stride(0))
            and (rscale is None or (rscale.is_contiguous() and rscale.dtype == torch.float32))):
        return False
    lib = nat.load()
    st = nat.stream(A.device)
    if X3_WSPLIT == "kernel" and B.data_ptr() % 16 == 0:
        # the weight split inside the GEMM while it is staged in LDS (no split launch, nothing cached)
        rc = lib.tmdnet_gemm_x3w_f32(M, N, K, A.data_ptr(), A.stride(0), B.data_ptr(), B.stride(0), int(bool(tb)),
                                     None if bias is None else bias.data_ptr(), C.data_ptr(), C.stride(0),
                                     int(bool(beta)), int(act), nat.ptr(pre), nat.ptr(rscale), nat.ptr(dpre),
                                     0 if x is None else x.stride(0), st)
        if rc != GEMM_UNSUPPORTED:
            nat.check(rc, "tmdnet_gemm_x3w_f32")
            return True
    bp = torch.empty((3, N, K), dtype=torch.int16, device=A.device)
    if tb:
        rc = lib.tmdnet_proj_split_f32(N, K, B.data_ptr(), B.stride(0), bp.data_ptr(), st)
    else:
        rc = lib.tmdnet_split_t_f32(N, K, B.data_ptr(), B.stride(0), bp.data_ptr(), st)
    if rc == GEMM_UNSUPPORTED:
        return False
    nat.check(rc, "tmdnet_split")
    rc = lib.tmdnet_gemm_x3_ex_f32(M, N, K, A.data_ptr(), A.stride(0), bp.data_ptr(),
                                   None if bias is None else bias.data_ptr(), C.data_ptr(), C.stride(0),
                                   int(bool(beta)), int(act), nat.ptr(pre), nat.ptr(rscale), nat.ptr(dpre),
                                   0 if x is None else x.stride(0), st)
    if rc == GEMM_UNSUPPORTED:
        return False
    nat.check(rc, "tmdnet_gemm_x3_ex_f32")
    return True


def gemm_group(problems):
    """The node feature-mix GEMMs of one step, grouped into one launch when the kernel supports
    them (fp32, up to GEMM_MAX_ROWS rows); large systems one tmdnet_gemm_x3_f32 launch each; otherwise
    the library GEMM (fp64 parity runs)."""
    if gemm_launch(problems):
        return
    mixed = len(problems) > 1
    for A, B, tb, bias, C, beta in problems:
        if A.shape[0] > GEMM_MAX_ROWS:
            if gemm_x3(A, B, tb, bias, C, beta):
                continue
        elif mixed and gemm_launch([(A, B, tb, bias, C, beta)]):  # (a group with rows on both sides)
            continue
        Bop = B.t() if tb else B
        if beta:
            C.addmm_(A, Bop)
            if bias is not None:
                C.add_(bias)
        elif bias is not None:
            torch.addmm(bias, A, Bop, out=C)
        else:
            torch.mm(A, Bop, out=C)


# ET dk/dv projection on the bf16 MFMA with an exact three-piece split (fp32 accuracy); TMDNET_PROJ=lib
# keeps the library fp32 GEMM (A/B switch)
PROJ = os.environ.get("TMDNET_PROJ", "x3")


def proj_split(W):
    """The exact three-piece bf16 split of a projection weight W [N, K] (``tmdnet_proj_split_f32``):
    an int16 tensor [3, N, K], or None when W is outside the kernel's envelope (then ``proj`` uses the
    library GEMM)."""
    N, K = W.shape
    if not (PROJ == "x3" and W.is_cuda and W.dtype == torch.float32 and W.stride(1) == 1 and K in (32, 64)
            and N % 16 == 0):
        return None
    wp = torch.empty((3, N, K), dtype=torch.int16, device=W.device)
    rc = nat.load().tmdnet_proj_split_f32(N, K, W.data_ptr(), W.stride(0), wp.data_ptr(), nat.stream(W.device))
    if rc == GEMM_UNSUPPORTED:
        return None
    nat.check(rc, "tmdnet_proj_split_f32")
    return wp


def proj(A, W, bias=None, out=None, wp=None, row0=0):
    """``A @ W.T (+ bias)`` for the dk/dv projection shapes (``tmdnet_proj_f32``: K = 32 / 64, fp32,
    16-byte aligned rows, N % 16 == 0); anything else, fp64 parity runs and ``TMDNET_PROJ=lib`` use
    the library GEMM on the same device.  ``wp``: W's split from ``proj_split`` when the caller shares
    it between GEMMs (W = rows [row0, row0 + N) of the split weight); ``out`` receives the result."""
    M, K = A.shape
    N = W.shape[0]
    if out is None:
        out = torch.empty((M, N), dtype=A.dtype, device=A.device)
    if (PROJ == "x3" and A.is_cuda and A.dtype == torch.float32 and A.stride(1) == 1 and out.stride(1) == 1
            and (bias is None or bias.is_contiguous())):
        if wp is None:
            wp, row0 = proj_split(W), 0
        if wp is not None:
            rc = nat.load().tmdnet_proj_f32(M, N, K, A.data_ptr(), A.stride(0), wp[0, row0:].data_ptr(),
                                            wp.shape[1] * K, None if bias is None else bias.data_ptr(),
                                            out.data_ptr(), out.stride(0), nat.stream(A.device))
            if rc != GEMM_UNSUPPORTED:
                nat.check(rc, "tmdnet_proj_f32")
                return out
    if bias is not None:
        return torch.addmm(bias, A, W.t(), out=out)
    return torch.mm(A, W.t(), out=out)


def wgrad_tn(problems):
    """Weight-gradient GEMMs C (+)= A^T B (+ A2^T B2), sums over the rows, all in one
    ``tmdnet_gemm_tn_f32`` launch (fp32; the library per problem otherwise).  Each problem is a dict:
    A [K, M], B [K, Nb] (or None with ``ones`` and C of one column), C [M, N], optional "beta",
    "ones" (C's last column = the column sums of A: B is implicitly [B | 1], N = Nb + 1), "A2" / "B2" /
    "ones2" (a second row segment of the same sum), "rows" (an int32 device scalar: only rows < rows of
    each segment are summed -- a static-capacity edge list's found pairs; the padding rows are zero)."""
    if not problems:
        return
    fp32 = all(p["A"].dtype == torch.float32 and p["A"].is_cuda for p in problems)
    if fp32:
        for i in range(0, len(problems), 32):
            _wgrad_tn_launch(problems[i:i + 32])
        return
    for p in problems:  # fp64 (parity runs): the library
        C, Cb = p["C"], p.get("Cb")
        ncol = C.shape[1] + int(Cb is not None)
        res = None
        for A, B, ones in ((p["A"], p.get("B"), p.get("ones", False)), (p.get("A2"), p.get("B2"), p.get("ones2", False))):
            if A is None or A.shape[0] == 0:
                continue
            Bx = B
            if ones:
                one = torch.ones((A.shape[0], 1), dtype=A.dtype, device=A.device)
                Bx = one if B is None else torch.cat((B, one), 1)
            elif B is not None and B.shape[1] < ncol:  # a second segment without the ones column
                Bx = torch.cat((B, torch.zeros((A.shape[0], 1), dtype=A.dtype, device=A.device)), 1)
            t = A.t() @ Bx
            res = t if res is None else res + t
        outs = [(C, res)] if Cb is None else [(C, res[:, :-1]), (Cb, res[:, -1])]
        for dst, val in outs:
            if p.get("beta"):
                dst.add_(val)
            else:
                dst.copy_(val)


def _wgrad_tn_launch(problems):
    lib = nat.load()
    n = len(problems)
    dims = (ctypes.c_int * (12 * n))()
    npp = 7 if any(p.get("rows") is not None for p in problems) else 6
    ptrs = (ctypes.c_void_p * (npp * n))()
    keep = []
    for i, p in enumerate(problems):
        A, B, C, Cb = p["A"], p.get("B"), p["C"], p.get("Cb")
        A2, B2 = p.get("A2"), p.get("B2")
        for t in (A, B, A2, B2, C, Cb):
            if t is not None and t.stride(-1) != 1:
                raise RuntimeError("wgrad_tn: operands need unit column stride")
        keep += [A, B, A2, B2, C, Cb]
        K2 = 0 if A2 is None else A2.shape[0]
        # with Cb, C holds the weight columns only: N counts the ones column too
        N = C.shape[1] + int(Cb is not None) if C.dim() == 2 else 1
        dims[12 * i:12 * i + 12] = [A.shape[1], N, A.shape[0], K2, A.stride(0),
                                    0 if B is None else B.stride(0), 0 if A2 is None else A2.stride(0),
                                    0 if B2 is None else B2.stride(0), C.stride(0) if C.dim() == 2 else 1,
                                    int(bool(p.get("beta"))), int(bool(p.get("ones"))), int(bool(p.get("ones2")))]
        rows = p.get("rows")
        if rows is not None and (rows.dtype != torch.int32 or rows.numel() != 1 or rows.device != A.device):
            raise RuntimeError("wgrad_tn: rows must be an int32 device scalar")
        ts = (A, B, A2, B2, C, Cb) + ((rows,) if npp == 7 else ())
        ptrs[npp * i:npp * i + npp] = [None if t is None else t.data_ptr() for t in ts]
    dev = problems[0]["A"].device
    wsb = lib.tmdnet_gemm_tn_workspace_bytes(n, dims)  # split over the rows: partial tiles
    ws = torch.empty((max(wsb, 4) // 4,), dtype=torch.float32, device=dev) if wsb else None
    fn = lib.tmdnet_gemm_tn_rows_f32_ws if npp == 7 else lib.tmdnet_gemm_tn_f32_ws
    rc = fn(n, dims, ptrs, None if ws is None else ws.data_ptr(), wsb, nat.stream(dev))
    nat.check(rc, "tmdnet_gemm_tn_f32_ws")


# ----------------------------------------------------------------------------- energy reduction
ATOM_SUM_MAX_MOLECULES = 8192


def _atom_sum_composite(x, batch, n_mol, std, mean):
    out = torch.zeros((n_mol,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device).index_add(0, batch, x * std)
    return out + mean


class _AtomSum(Function):
    """y[b] = mean + std * sum_{batch[n] = b} x[n] (TorchMD_Net.forward: `x * std`, reduce, `+ mean`)."""

    @staticmethod
    def forward(ctx, x, batch, n_mol, std, mean):
        lib = nat.load()
        y = torch.empty((n_mol, 1), dtype=x.dtype, device=x.device)
        rc = lib.tmdnet_atom_sum_fwd(nat.dtype_code(x.dtype), x.shape[0], n_mol, nat.ptr(x), nat.ptr(batch),
                                     nat.ptr(std), nat.ptr(mean), nat.ptr(y), nat.stream(x.device))
        nat.check(rc, "tmdnet_atom_sum_fwd")
        ctx.n_mol = n_mol
        ctx.save_for_backward(batch, std)
        return y

    @staticmethod
    def backward(ctx, gy):
        batch, std = ctx.saved_tensors
        return _AtomSumBwd.apply(gy.contiguous(), batch, std, ctx.n_mol), None, None, None, None


class _AtomSumBwd(Function):
    @staticmethod
    def forward(ctx, gy, batch, std, n_mol):
        lib = nat.load()
        gx = torch.empty((batch.shape[0], 1), dtype=gy.dtype, device=gy.device)
        rc = lib.tmdnet_atom_sum_bwd(nat.dtype_code(gy.dtype), batch.shape[0], n_mol, nat.ptr(gy), nat.ptr(batch),
                                     nat.ptr(std), nat.ptr(gx), nat.stream(gy.device))
        nat.check(rc, "tmdnet_atom_sum_bwd")
        ctx.n_mol = n_mol
        ctx.save_for_backward(batch, std)
        return gx

    @staticmethod
    def backward(ctx, ggx):  # linear in gy: its adjoint is the reduction again (std a buffer)
        batch, std = ctx.saved_tensors
        return _atom_sum_composite(ggx, batch, ctx.n_mol, std, torch.zeros_like(std)), None, None, None


def atom_sum(x, batch, n_mol, std, mean):
    """Fused ``reduce(x * std) + mean`` of TorchMD_Net.forward for a [N, 1] per-atom output."""
    nat.require_gpu(x, "atom_sum")
    return _AtomSum.apply(x.contiguous(), batch, int(n_mol), std, mean)


def _dot_sum_launch(h, w, b0, batch, n_mol, std, mean):
    """y[b] = mean + std * sum_{batch[n] = b} (h[n] . w + b0), one tmdnet_dot_sum_fwd_atoms launch."""
    y = torch.empty((n_mol, 1), dtype=h.dtype, device=h.device)
    # large systems: the row products over the whole grid first (per-atom buffer)
    buf = torch.empty(h.shape[0], dtype=h.dtype, device=h.device) if h.shape[0] > 4096 else None
    rc = nat.load().tmdnet_dot_sum_fwd_atoms(nat.dtype_code(h.dtype), h.shape[0], h.shape[1], nat.ptr(h), h.stride(0),
                                             nat.ptr(w), nat.ptr(b0), n_mol, nat.ptr(batch), nat.ptr(std),
                                             nat.ptr(mean), nat.ptr(buf), nat.ptr(y), nat.stream(h.device))
    nat.check(rc, "tmdnet_dot_sum_fwd")
    return y


def _dot_sum_bwd_launch(gy, batch, n_mol, std, w, rows):
    """gh[n] = std * gy[batch[n]] * w (tmdnet_dot_sum_bwd), [rows, len(w)]."""
    gh = torch.empty((rows, w.shape[0]), dtype=gy.dtype, device=gy.device)
    rc = nat.load().tmdnet_dot_sum_bwd(nat.dtype_code(gy.dtype), rows, w.shape[0], nat.ptr(gy), nat.ptr(batch), n_mol,
                                       nat.ptr(std), nat.ptr(w), nat.ptr(gh), nat.stream(gy.device))
    nat.check(rc, "tmdnet_dot_sum_bwd")
    return gh


def _dot_sum_composite(h, w, b0, batch, n_mol, std, mean):
    x = h @ w.view(-1, 1) + b0.view(1, 1)
    return _atom_sum_composite(x, batch, n_mol, std, mean)


class _DotSum(Function):
    """y[b] = mean + std * sum_{batch[n] = b} (h[n] . w + b0): the Scalar head's last Linear (H/2 -> 1)
    fused with TorchMD_Net's `x * std`, per-molecule sum and `+ mean` (tmdnet_dot_sum_fwd)."""

    @staticmethod
    def forward(ctx, h, w, b0, batch, n_mol, std, mean):
        y = _dot_sum_launch(h, w, b0, batch, n_mol, std, mean)
        ctx.n_mol = n_mol
        ctx.save_for_backward(h, w, b0, batch, std)
        return y

    @staticmethod
    def backward(ctx, gy):
        h, w, b0, batch, std = ctx.saved_tensors
        nf = ctx.next_functions
        need = (ctx.needs_input_grad[0] and _will_run(nf[0][0]), ctx.needs_input_grad[1] and _will_run(nf[1][0]),
                ctx.needs_input_grad[2] and _will_run(nf[2][0]))
        if not any(need):
            return None, None, None, None, None, None, None
        gh, gw, gb = _DotSumBwd.apply(gy.contiguous(), h, w, b0, batch, std, ctx.n_mol, need)
        return gh, gw, gb, None, None, None, None


class _DotSumBwd(Function):
    @staticmethod
    def forward(ctx, gy, h, w, b0, batch, std, n_mol, need):
        gh = gw = gb = None
        if need[0]:
            gh = _dot_sum_bwd_launch(gy, batch, n_mol, std, w, h.shape[0])
        if need[1] or need[2]:  # training: the per-atom seed a = std * gy[batch], then (a^T h, sum a): one TN launch
            ga = (std * gy.index_select(0, batch).view(-1)).view(-1, 1)
            gw, gb = _linear_wgrad(ga, h, need[1], need[2])
            gw = gw.view(-1) if gw is not None else None
        ctx.n_mol = n_mol
        ctx.save_for_backward(gy, h, w, b0, batch, std)
        return gh, gw, gb

    @staticmethod
    def backward(ctx, ggh, ggw, ggb):
        gy, h, w, b0, batch, std = ctx.saved_tensors
        n_mol = ctx.n_mol
        zero = torch.zeros_like(std)
        if h.is_cuda and h.dtype == torch.float32 and not torch.is_grad_enabled():
            # hand VJP of (gh = a w, gw = a^T h, gb = sum a), a_n = std gy[batch[n]]:
            #   d_gy[b] = std sum_{batch[n] = b} (ggh[n] . w + h[n] . ggw + ggb),
            #   d_h = a ggw,  d_w = a^T ggh  (no library GEMM: dot-sum / TN launches)
            d_gy = None
            if ggh is not None or ggb is not None:
                d_gy = _dot_sum_launch(ggh if ggh is not None else torch.zeros_like(h), w,
                                       ggb.reshape(1) if ggb is not None else zero.reshape(1), batch, n_mol, std, zero)
            if ggw is not None:
                t = _dot_sum_launch(h, ggw.reshape(-1), zero.reshape(1), batch, n_mol, std, zero)
                d_gy = t if d_gy is None else d_gy + t
            d_h = _dot_sum_bwd_launch(gy, batch, n_mol, std, ggw.reshape(-1), h.shape[0]) if ggw is not None else None
            d_w = None
            if ggh is not None:
                ga = (std * gy.index_select(0, batch).view(-1)).view(-1, 1)
                d_w = _linear_wgrad(ga, ggh.contiguous(), True, False)[0].view(-1)
            return d_gy, d_h, d_w, None, None, None, None, None
        # (fp64 / a graph of the second order: the composite differentiated twice)
        d = _tn_double_backward(lambda h_, w_, b_: _dot_sum_composite(h_, w_, b_, batch, n_mol, std, zero),
                                [h, w, b0], [gy], [ggh, ggw, ggb])
        return d[0], d[1], d[2], d[3], None, None, None, None


def dot_sum(h, w, b0, batch, n_mol, std, mean):
    """Fused ``reduce((h w + b0) * std) + mean`` (Scalar head's last Linear + TorchMD_Net's reduction)."""
    nat.require_gpu(h, "dot_sum")
    return _DotSum.apply(h.contiguous(), w.reshape(-1), b0.reshape(-1), batch, int(n_mol), std, mean)


# ----------------------------------------------------------------------------- TensorNet
def _self0_args(graph):
    """(host multiplicity, device pair count, padding capacity) for the TN kernels' atom-0 self loop
    (static_shapes emulation).  ``graph.self0_dev`` = (num_pairs tensor, capacity) selects the
    device-side form used under HIP-graph capture."""
    dev = getattr(graph, "self0_dev", None)
    if dev is not None:
        return 1.0, nat.ptr(dev[0]), int(dev[1])
    return float(getattr(graph, "self0_mult", 1.0)), None, 0


def _self0_weight(graph, like):
    w = torch.ones(graph.n_edges, dtype=like.dtype, device=like.device)
    dev = getattr(graph, "self0_dev", None)
    if dev is not None:
        m = (1 + (dev[1] - dev[0].to(torch.int64)).clamp(min=0)).to(like.dtype)
        return torch.where((graph.src == 0) & (graph.dst == 0), m.expand_as(w), w)
    m = getattr(graph, "self0_mult", 1.0)
    if m != 1.0:
        w = torch.where((graph.src == 0) & (graph.dst == 0), torch.full_like(w, m), w)
    return w


def _skew(v):
    z = torch.zeros_like(v[:, 0])
    return torch.stack((z, -v[:, 2], v[:, 1], v[:, 2], z, -v[:, 0], -v[:, 1], v[:, 0], z), dim=1).view(-1, 3, 3)


def _sym(v):
    t = v.unsqueeze(-1) * v.unsqueeze(-2)
    eye = torch.eye(3, dtype=v.dtype, device=v.device)
    return 0.5 * (t + t.transpose(-2, -1)) - t.diagonal(dim1=-2, dim2=-1).mean(-1)[..., None, None] * eye


def _skew_c(u):
    """compact coordinates (a01, a02, a12) of skew(u) (tensornet.py:16-34)."""
    return torch.stack((-u[:, 2], u[:, 1], -u[:, 0]), dim=1)


def _sym_c(u):
    """compact coordinates (s00, s11, s01, s02, s12) of sym(u) = u u^T - |u|^2/3 Id (tensornet.py:37-44)."""
    tr = (u * u).sum(1) / 3
    return torch.stack((u[:, 0] * u[:, 0] - tr, u[:, 1] * u[:, 1] - tr, u[:, 0] * u[:, 1],
                        u[:, 0] * u[:, 2], u[:, 1] * u[:, 2]), dim=1)


def tn_embed_composite(P, Q, W, C, u, graph):
    """tensornet.py:295-315 in reference orientation (scatter to edge_index[0]); compact [9, N, H]."""
    valid = (graph.src >= 0).to(P.dtype)  # static-capacity padding slots (-1) carry nothing
    src, dst = graph.src.long().clamp(min=0), graph.dst.long().clamp(min=0)
    H = P.shape[1]
    N = graph.n_nodes
    wt = (_self0_weight(graph, C) * C * valid).unsqueeze(1)
    z = (P.index_select(0, src) + Q.index_select(0, dst)) * wt
    W1, W2, W3 = W[:, :H], W[:, H:2 * H], W[:, 2 * H:]
    coef = [z * W1] + [(z * W2) * a.unsqueeze(1) for a in _skew_c(u).unbind(1)] \
        + [(z * W3) * s.unsqueeze(1) for s in _sym_c(u).unbind(1)]
    zero = torch.zeros((N, H), dtype=P.dtype, device=P.device)
    return torch.stack([zero.index_add(0, src, c) for c in coef], dim=0)


def tn_message_composite(ea, Tc, graph):
    """tensornet.py:329-332 (gather edge_index[1], scatter edge_index[0]) on compact [9, N, H] tensors."""
    valid = (graph.src >= 0).to(Tc.dtype)
    src, dst = graph.src.long().clamp(min=0), graph.dst.long().clamp(min=0)
    N, H = Tc.shape[1], Tc.shape[2]
    f = (ea.reshape(-1, H, 3) * (_self0_weight(graph, ea) * valid).view(-1, 1, 1))
    zero = torch.zeros((N, H), dtype=Tc.dtype, device=Tc.device)
    rows = [zero.index_add(0, src, f[..., 0 if k == 0 else (1 if k < 4 else 2)] * Tc[k].index_select(0, dst))
            for k in range(9)]
    return torch.stack(rows, dim=0)


def tn_embed_fwd_launch(P, Q, W, C, u, graph, out):
    lib = nat.load()
    N, H = P.shape
    rc = lib.tmdnet_tn_embed_fwd(nat.dtype_code(P.dtype), N, H, nat.ptr(graph.row_ptr), nat.ptr(graph.src),
                                 graph.n_edges, *_self0_args(graph), nat.ptr(P), nat.ptr(Q), nat.ptr(W), _ld(W),
                                 nat.ptr(C), nat.ptr(u), nat.ptr(out), nat.stream(P.device))
    nat.check(rc, "tmdnet_tn_embed_fwd")


def tn_embed_bwd_launch(P, Q, W, C, u, graph, gE, gP, gQ, gW, gC, gu):
    lib = nat.load()
    N, H = P.shape
    rc = lib.tmdnet_tn_embed_bwd(nat.dtype_code(P.dtype), N, H, nat.ptr(graph.row_ptr), nat.ptr(graph.src),
                                 graph.n_edges, *_self0_args(graph), nat.ptr(P), nat.ptr(Q), nat.ptr(W), _ld(W),
                                 nat.ptr(C), nat.ptr(u), nat.ptr(gE), nat.ptr(gP), nat.ptr(gQ), nat.ptr(gW),
                                 nat.ptr(gC), nat.ptr(gu), nat.stream(P.device))
    nat.check(rc, "tmdnet_tn_embed_bwd")


def tn_message_fwd_launch(ea, Tc, graph, out, pairs=None):
    """``pairs`` = (pair_row [E], pair_edge [P]) of ``pair_index``: ea holds one row per pair slot."""
    lib = nat.load()
    N, H = Tc.shape[1], Tc.shape[2]
    if pairs is not None:
        rc = lib.tmdnet_tn_message_fwd_pairs(nat.dtype_code(Tc.dtype), N, H, nat.ptr(graph.row_ptr),
                                             nat.ptr(graph.src), graph.n_edges, *_self0_args(graph),
                                             nat.ptr(pairs[0]), nat.ptr(ea), _ld(ea), nat.ptr(Tc), nat.ptr(out),
                                             nat.stream(Tc.device))
        nat.check(rc, "tmdnet_tn_message_fwd_pairs")
        return
    rc = lib.tmdnet_tn_message_fwd(nat.dtype_code(Tc.dtype), N, H, nat.ptr(graph.row_ptr), nat.ptr(graph.src),
                                   graph.n_edges, *_self0_args(graph), nat.ptr(ea), _ld(ea), nat.ptr(Tc),
                                   nat.ptr(out), nat.stream(Tc.device))
    nat.check(rc, "tmdnet_tn_message_fwd")


def tn_message_bwd_launch(ea, Tc, graph, gmsg, gea, gT, gadd=None, pairs=None):
    lib = nat.load()
    N, H = Tc.shape[1], Tc.shape[2]
    if pairs is not None:
        rc = lib.tmdnet_tn_message_bwd_pairs(nat.dtype_code(Tc.dtype), N, H, nat.ptr(graph.row_ptr),
                                             nat.ptr(graph.src), graph.n_edges, *_self0_args(graph),
                                             nat.ptr(pairs[0]), nat.ptr(pairs[1]), pairs[1].shape[0], nat.ptr(ea),
                                             _ld(ea), nat.ptr(Tc), nat.ptr(gmsg), nat.ptr(gadd), nat.ptr(gea),
                                             nat.ptr(gT), nat.stream(Tc.device))
        nat.check(rc, "tmdnet_tn_message_bwd_pairs")
        return
    rc = lib.tmdnet_tn_message_bwd_add(nat.dtype_code(Tc.dtype), N, H, nat.ptr(graph.row_ptr), nat.ptr(graph.src),
                                       graph.n_edges, *_self0_args(graph), nat.ptr(ea), _ld(ea), nat.ptr(Tc),
                                       nat.ptr(gmsg), nat.ptr(gadd), nat.ptr(gea), nat.ptr(gT), nat.stream(Tc.device))
    nat.check(rc, "tmdnet_tn_message_bwd_add")


def _ea_edges(ea, pairs):
    """Per-edge factor rows from pair rows (differentiable gather; the composite restatements)."""
    return ea if pairs is None else ea.index_select(0, pairs[0].long())


class _TNEmbed(Function):
    @staticmethod
    def forward(ctx, P, Q, W, C, u, graph):
        N, H = P.shape
        out = torch.empty((9, N, H), dtype=P.dtype, device=P.device)
        tn_embed_fwd_launch(P, Q, W, C, u, graph, out)
        ctx.graph = graph
        ctx.save_for_backward(P, Q, W, C, u)
        return out

    @staticmethod
    def backward(ctx, gE):
        P, Q, W, C, u = ctx.saved_tensors
        outs = _TNEmbedBwd.apply(gE.contiguous(), P, Q, W, C, u, ctx.graph)
        return tuple(outs) + (None,)


class _TNEmbedBwd(Function):
    @staticmethod
    def forward(ctx, gE, P, Q, W, C, u, graph):
        if not graph.symmetric:
            raise RuntimeError("torchmd-net_amd: TensorNet backward needs a symmetric edge list")
        N, H = P.shape
        E = graph.n_edges
        o = dict(dtype=P.dtype, device=P.device)
        gP, gQ = torch.empty((N, H), **o), torch.empty((N, H), **o)
        gW = torch.empty((E, 3 * H), **o)
        gC, gu = torch.empty((E,), **o), torch.empty((E, 3), **o)
        tn_embed_bwd_launch(P, Q, W, C, u, graph, gE, gP, gQ, gW, gC, gu)
        ctx.graph = graph
        ctx.save_for_backward(gE, P, Q, W, C, u)
        return gP, gQ, gW, gC, gu

    @staticmethod
    def backward(ctx, *ggs):
        saved = ctx.saved_tensors
        _create = torch.is_grad_enabled()  # third order only if the caller builds a graph
        from . import tn_node
        if tn_node.SECOND_ORDER != "composite" and not _create and saved[0].is_cuda:
            return _tn_embed_second_order(ctx, saved, ggs)
        with torch.enable_grad():
            leaves = [t.detach().requires_grad_(True) for t in saved]
            gE, P, Q, W, C, u = leaves
            E_ = tn_embed_composite(P, Q, W, C, u, ctx.graph)
            first = torch.autograd.grad(E_, (P, Q, W, C, u), gE, create_graph=True)
            sel = [(f, g) for f, g in zip(first, ggs) if g is not None]
            if not sel:
                return (None,) * 7
            second = torch.autograd.grad([f for f, _ in sel], leaves, [g for _, g in sel],
                                         create_graph=_create, allow_unused=True)
        return tuple(second) + (None,)


def _tn_embed_second_order(ctx, saved, ggs):
    """VJP of the embedding's first backward (gP, gQ, gW, gC, gu) = J^T gE for cotangents t of those outputs:
    d_gE = J t and d_(P, Q, W, C, u) = H_<gE, E> t -- ONE tmdnet_tn_embed_bwd2 call (the first-order kernels on
    dual numbers) instead of autograd's double differentiation of the composite (~370 launches per C3 step)."""
    gE, P, Q, W, C, u = saved
    graph = ctx.graph
    need = ctx.needs_input_grad  # gE, P, Q, W, C, u, graph
    t = [None if g is None else g.contiguous() for g in ggs]
    if all(x is None for x in t):
        return (None,) * 7
    tW = t[2]
    if tW is not None and tW.stride(0) != W.stride(0):
        W = W.contiguous()
        tW = tW.contiguous()
    o = dict(dtype=P.dtype, device=P.device)
    N, H = P.shape
    E = graph.n_edges
    outs = [torch.empty((9, N, H), **o) if need[0] else None,
            torch.empty((N, H), **o) if need[1] else None, torch.empty((N, H), **o) if need[2] else None,
            torch.empty((E, 3 * H), **o) if need[3] else None, torch.empty((E,), **o) if need[4] else None,
            torch.empty((E, 3), **o) if need[5] else None]
    lib = nat.load()
    rc = lib.tmdnet_tn_embed_bwd2(nat.dtype_code(P.dtype), N, H, nat.ptr(graph.row_ptr), nat.ptr(graph.src),
                                  graph.n_edges, *_self0_args(graph), nat.ptr(P), nat.ptr(Q), nat.ptr(W), _ld(W),
                                  nat.ptr(C), nat.ptr(u), nat.ptr(gE), *[nat.ptr(x) for x in (t[0], t[1], tW, t[3], t[4])],
                                  *[nat.ptr(x) for x in outs], nat.stream(P.device))
    nat.check(rc, "tmdnet_tn_embed_bwd2")
    return tuple(outs) + (None,)


class _TNMessage(Function):
    """The message.  ``fanout``: also returns an alias of Tc for its second consumer (the POST pass); that
    consumer's gradient is added by the message backward kernel (no separate add launch).  ``pairs``: ea is
    given per pair slot (``pair_index``), its gradient likewise."""

    @staticmethod
    def forward(ctx, ea, Tc, graph, fanout, pairs=None):
        msg = torch.empty_like(Tc)
        tn_message_fwd_launch(ea, Tc, graph, msg, pairs)
        ctx.graph = graph
        ctx.pairs = pairs
        ctx.save_for_backward(ea, Tc)
        if fanout:
            return msg, Tc.view_as(Tc)
        return msg

    @staticmethod
    def backward(ctx, gmsg, galias=None):
        ea, Tc = ctx.saved_tensors
        if gmsg is None:
            gmsg = torch.zeros_like(Tc)
        gadd = None if galias is None else galias.contiguous()
        outs = _TNMessageBwd.apply(gmsg.contiguous(), ea, Tc, ctx.graph, gadd, ctx.pairs)
        return tuple(outs) + (None, None, None)


class _TNMessageBwd(Function):
    @staticmethod
    def forward(ctx, gmsg, ea, Tc, graph, gadd, pairs=None):
        if not graph.symmetric:
            raise RuntimeError("torchmd-net_amd: TensorNet backward needs a symmetric edge list")
        H = Tc.shape[2]
        gea = torch.empty((ea.shape[0], 3 * H), dtype=Tc.dtype, device=Tc.device)
        gT = torch.empty_like(Tc)
        tn_message_bwd_launch(ea, Tc, graph, gmsg, gea, gT, gadd, pairs)
        ctx.graph = graph
        ctx.pairs = pairs
        ctx.has_add = gadd is not None
        ctx.save_for_backward(gmsg, ea, Tc)
        return gea, gT

    @staticmethod
    def backward(ctx, *ggs):
        saved = ctx.saved_tensors
        _create = torch.is_grad_enabled()  # third order only if the caller builds a graph
        g_add = ggs[1] if ctx.has_add else None  # gT = VJP(gmsg) + gadd: identity in gadd
        from . import tn_node
        if tn_node.SECOND_ORDER != "composite" and not _create:
            return _tn_message_second_order(ctx, saved, ggs) + (None, g_add, None)
        with torch.enable_grad():
            leaves = [t.detach().requires_grad_(True) for t in saved]
            gmsg, ea, Tc = leaves
            msg = tn_message_composite(_ea_edges(ea, ctx.pairs), Tc, ctx.graph)
            first = torch.autograd.grad(msg, (ea, Tc), gmsg, create_graph=True)
            sel = [(f, g) for f, g in zip(first, ggs) if g is not None]
            if not sel:
                return (None,) * 4 + (g_add, None)
            second = torch.autograd.grad([f for f, _ in sel], leaves, [g for _, g in sel],
                                         create_graph=_create, allow_unused=True)
        return tuple(second) + (None, g_add, None)


def _tn_message_second_order(ctx, saved, ggs):
    """The message is bilinear in (ea, Tc): with (gea, gT) = (G(gmsg, Tc), M^T(ea, gmsg)) its second-order
    VJP for cotangents (t_ea, t_T) is d_gmsg = M(t_ea, Tc) + M(ea, t_T) (two forward launches) and
    (d_ea, d_T) = (G(gmsg, t_T), M^T(t_ea, gmsg)) -- ONE first-backward launch with (t_ea, t_T) in place of
    (ea, Tc).  The first backward's pair-symmetry precondition then applies to t_ea: the edge factors'
    cotangent is, like the factors, a function of the pair distance (edge MLP -> rbf -> r, whose
    cotangent <t_pos[src] - t_pos[dst], u> is the same for both directions of a pair).  (Pair rows: t_ea is
    per pair slot, the same kernels with pair_row.)"""
    gmsg, ea, Tc = saved
    t_ea, t_T = ggs
    graph = ctx.graph
    pairs = ctx.pairs
    need = ctx.needs_input_grad  # gmsg, ea, Tc, graph, gadd
    if t_ea is None and t_T is None:
        return None, None, None
    t_ea = torch.zeros_like(ea) if t_ea is None else _rowmajor(t_ea)
    t_T = torch.zeros_like(Tc) if t_T is None else t_T.contiguous()
    d_g = None
    if need[0]:
        d_g = torch.empty_like(Tc)
        tn_message_fwd_launch(t_ea, Tc, graph, d_g, pairs)
        tmp = torch.empty_like(Tc)
        tn_message_fwd_launch(ea, t_T, graph, tmp, pairs)
        d_g.add_(tmp)
    d_ea = d_T = None
    if need[1] or need[2]:
        d_ea = torch.empty((ea.shape[0], 3 * Tc.shape[2]), dtype=Tc.dtype, device=Tc.device)
        d_T = torch.empty_like(Tc)
        tn_message_bwd_launch(t_ea, t_T, graph, gmsg, d_ea, d_T, pairs=pairs)
    return d_g, (d_ea if need[1] else None), (d_T if need[2] else None)


def tn_embed(P, Q, W, C, u, graph):
    """Embedding aggregation -> compact [9, N, H] (I | A | S rows)."""
    nat.require_gpu(P, "tn_embed")
    return _TNEmbed.apply(P.contiguous(), Q.contiguous(), _rowmajor(W), C.contiguous(), u.contiguous(), graph)


def tn_message(ea, Tc, graph, fanout=False, pairs=None):
    """Tensor message passing on a compact [9, N, H] tensor -> compact message (``fanout``: and an alias
    of Tc for its second consumer, whose gradient the message backward adds).  ``pairs`` = ``pair_index``'s
    (pair_row, pair_edge): ea has one row per pair slot (large systems: the edge MLP runs per pair)."""
    nat.require_gpu(Tc, "tn_message")
    return _TNMessage.apply(_rowmajor(ea), Tc.contiguous(), graph, fanout, pairs)


# ----------------------------------------------------------------------------- spatial order
REORDER_MIN_ATOMS = 16384


def _spread10(x):
    x = x & 0x3FF
    x = (x | (x << 16)) & 0x030000FF
    x = (x | (x << 8)) & 0x0300F00F
    x = (x | (x << 4)) & 0x030C30C3
    x = (x | (x << 2)) & 0x09249249
    return x


def spatial_permutation(pos, batch, cell_size, box=None):
    """Permutation that renumbers atoms molecule-major, then by the Morton (Z-order) index of their
    cutoff-sized cell.  Edge kernels gather source rows of spatial neighbours; with this numbering
    the waves in flight on one XCD touch a compact window of rows (L2 reuse): +25-30 % on the
    C5 water box vs random numbering (tools/kbench.py).  Sync-free (device argsort)."""
    p = pos.detach()
    if box is not None and box.numel() == 9:
        # the box lives in host memory (reference OptimizedDistance keeps it on the CPU): its diagonal as
        # Python scalars, so no host-to-device copy is issued (not allowed inside a graph capture)
        L = torch.diagonal(box.detach().cpu()).tolist()
        p = torch.stack([torch.remainder(p[:, i], float(L[i])) for i in range(3)], dim=1)
    lo = p.min(dim=0).values
    c = torch.clamp(((p - lo) / float(cell_size)).long(), 0, 1023)
    key = _spread10(c[:, 0]) | (_spread10(c[:, 1]) << 1) | (_spread10(c[:, 2]) << 2)
    key = key + batch.to(torch.long) * (1 << 31)
    return torch.argsort(key, stable=True)


# ----------------------------------------------------------------------------- EquivariantScalar head
def eq_head_params(blocks):
    """The 12 tensors tmdnet_eq_head_fwd consumes, in its order (include/tmdnet.h)."""
    ps = []
    for b in blocks:
        ps += [b.vec1_proj.weight, b.vec2_proj.weight, b.update_net[0].weight, b.update_net[0].bias,
               b.update_net[2].weight, b.update_net[2].bias]
    return ps


def eq_head_fusable(blocks):
    """Two GatedEquivariantBlocks H -> H/2 (scalar SiLU) -> 1, SiLU update nets, intermediate = hidden
    (EquivariantScalar's configuration, reference output_modules.py:80-100)."""
    if len(blocks) != 2:
        return False
    b1, b2 = blocks
    H = b1.vec1_proj.in_features
    shapes_ok = (H % 4 == 0 and b1.out_channels == H // 2 and b2.out_channels == 1
                 and b2.vec1_proj.in_features == H // 2
                 and b1.update_net[0].out_features == H and b2.update_net[0].out_features == H // 2)
    acts_ok = all(isinstance(b.update_net[1], torch.nn.SiLU) for b in blocks) \
        and isinstance(b1.act, torch.nn.SiLU) and b2.act is None
    return bool(shapes_ok and acts_ok and all(b.update_net[0].bias is not None for b in blocks))


def masked_norm(vb):
    """|vb| over the axis dim (-2) with the reference's zero-row exclusion (utils.py:500-512:
    rows whose vectors are all zero keep 0 and get no gradient of any order), sync-free."""
    nz = (vb != 0).flatten(1).any(dim=1).view(-1, 1, 1)
    nrm = torch.linalg.vector_norm(torch.where(nz, vb, torch.ones_like(vb)), dim=-2)
    return torch.where(nz.view(-1, 1), nrm, torch.zeros_like(nrm))


def eq_head_composite(x, vec, params):
    """Differentiable restatement of the two gated blocks (reference utils.py:492-522): the vector
    norm's gradient is 0 where the norm is 0 (the reference masks zero rows, utils.py:500-512)."""
    for blk, scalar_act in ((0, True), (1, False)):
        w1, w2, u1w, u1b, u2w, u2b = params[6 * blk:6 * blk + 6]
        vec1 = masked_norm(torch.matmul(vec, w1.t()))
        vec2 = torch.matmul(vec, w2.t())
        o = F.linear(F.silu(F.linear(torch.cat([x, vec1], dim=-1), u1w, u1b)), u2w, u2b)
        xo, vo = torch.split(o, w2.shape[0], dim=-1)
        vec = vo.unsqueeze(1) * vec2
        x = F.silu(xo) if scalar_act else xo
    return x + vec.sum() * 0  # keeps every parameter in the graph (zero, not None, gradients)


def _will_run(node):
    if node is None:
        return False
    try:
        return bool(torch._C._will_engine_execute_node(node))
    except RuntimeError:
        return True


# the head's forward + Jacobian on the bf16 MFMA over 16-atom tiles (tmdnet_eq_head_x3_f32; fp32, H = 128);
# TMDNET_HEAD_X3=0: the per-atom VALU kernel (A/B).  Below HEAD_X3_MIN_ATOMS the per-atom kernel is the
# faster one (tools/head_ab.py, graph-replayed fwd + Jacobian: 678 atoms 40.2 µs VALU vs 47.4 MFMA;
# 1024 atoms 59.1 vs 47.5; 50000 atoms 1255 vs 549)
HEAD_X3 = os.environ.get("TMDNET_HEAD_X3", "1") != "0"
HEAD_X3_MIN_ATOMS = int(os.environ.get("TMDNET_HEAD_X3_MIN_ATOMS", "768"))


def _eq_head_x3(lib, x, vec, params, y, jx, jv):
    """tmdnet_eq_head_x3_split_f32 (the weights' pieces, one launch: they always match the current weights,
    also inside a captured step) + tmdnet_eq_head_x3_f32.  Returns False outside its envelope."""
    N, H = x.shape
    nbytes = int(lib.tmdnet_eq_head_x3_pieces_bytes(H))
    if not (HEAD_X3 and N >= HEAD_X3_MIN_ATOMS and nbytes and x.dtype == torch.float32 and all(p.is_contiguous() for p in params)
            and all(p.data_ptr() % 16 == 0 for p in (params[3], params[5], params[9]))):
        return False
    st = nat.stream(x.device)
    buf = torch.empty((nbytes // 2,), dtype=torch.int16, device=x.device)
    ws = (ctypes.c_void_p * 12)(*[p.data_ptr() for p in params])
    rc = lib.tmdnet_eq_head_x3_split_f32(H, ws, buf.data_ptr(), st)
    if rc == GEMM_UNSUPPORTED:
        return False
    nat.check(rc, "tmdnet_eq_head_x3_split_f32")
    O = H // 2
    nk = [(H + O, H), (H, 2 * H), (H, H), (O, O), (O, 2 * O), (2 * O, O), (O, O), (H, H), (2 * H, H), (H, H + O)]
    offs, o = [], 0
    for n, k in nk:
        offs.append(buf.data_ptr() + 2 * o)
        o += 3 * n * k
    pieces = (ctypes.c_void_p * 10)(*offs)
    vecs = (ctypes.c_void_p * 5)(*[params[i].data_ptr() for i in (3, 5, 9, 10, 11)])
    rc = lib.tmdnet_eq_head_x3_f32(N, H, nat.ptr(x), nat.ptr(vec), pieces, vecs, nat.ptr(y), nat.ptr(jx),
                                   nat.ptr(jv), None, st)
    nat.check(rc, "tmdnet_eq_head_x3_f32")
    return True


class _EqHead(Function):
    """(x, vec, *head params) -> y [N, 1]; the HIP kernel also returns dy/dx, dy/dvec per atom."""

    @staticmethod
    def forward(ctx, x, vec, *params):
        lib = nat.load()
        N, H = x.shape
        x, vec = x.contiguous(), vec.contiguous()
        y = torch.empty((N, 1), dtype=x.dtype, device=x.device)
        want_j = ctx.needs_input_grad[0] or ctx.needs_input_grad[1]
        jx = torch.empty_like(x) if want_j else None
        jv = torch.empty_like(vec) if want_j else None
        if not (N and _eq_head_x3(lib, x, vec, params, y, jx, jv)):
            ws = (ctypes.c_void_p * 12)(*[p.data_ptr() for p in params])
            rc = lib.tmdnet_eq_head_fwd(nat.dtype_code(x.dtype), N, H, nat.ptr(x), nat.ptr(vec), ws, nat.ptr(y),
                                        nat.ptr(jx), nat.ptr(jv), nat.stream(x.device))
            nat.check(rc, "tmdnet_eq_head_fwd")
        ctx.save_for_backward(x, vec, jx, jv, *params)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, vec, jx, jv, *params = ctx.saved_tensors
        nf = ctx.next_functions
        off = len(nf) - len(params)
        need_w = any(_will_run(nf[off + i][0]) for i in range(len(params)))
        # a force-matching loss backward reaches the head twice (here and its force pass's HVP): see _HeadLink
        # (the HVP takes part only in its hand-written form: no third order, not the composite switch)
        hand_ok = need_w and HEAD_HANDOFF and not torch.is_grad_enabled() and HEAD_SECOND_ORDER != "composite"
        link = getattr(ctx, "link", None) if hand_ok else None
        seg2 = link.take("fwd") if link is not None else None
        stash = link if (link is not None and seg2 is None and link.other_will_run("fwd")) else None
        outs = _EqHeadBwd.apply((need_w, seg2, stash), gy.contiguous(), jx, jv, x, vec, *params)
        if outs[0].grad_fn is not None:  # (create_graph: the force pass)
            link = _HeadLink(weakref.ref(ctx), weakref.ref(outs[0].grad_fn))
            ctx.link = link
            outs[0].grad_fn.link = link
        return outs


def _head_factor_ops(n, H, a1, vv, gu, hext, go, sext, a2, v1, gu2, h2ext, go2, s2ext):
    O = Q = H // 2
    return [(a1.view(3 * n, H + O), vv.reshape(3 * n, H)), (gu, hext), (go, sext),
            (a2.view(3 * n, Q + 1), v1.view(3 * n, O)), (gu2, h2ext), (go2, s2ext)]


def _head_wgrads(n, H, *factors, seg2=None):
    """The head's six weight-gradient GEMMs over the n per-atom factor rows, in one grouped launch;
    ``seg2`` = (n2, factors2): a second set of factor rows summed by the same GEMMs (the other pass's).
    Returns the 12 parameter gradients, each contiguous (a bias is its factor's last column, written to
    its own vector: no strided column blocks for the training step's gradient copy)."""
    O = Q = H // 2
    a1 = factors[0]
    o = dict(dtype=a1.dtype, device=a1.device)
    e = lambda *shape: torch.empty(shape, **o)  # noqa: E731
    w12, v12 = e(H + O, H), e(Q + 1, O)
    u1, u1b, u2, u2b = e(H, 2 * H), e(H), e(2 * O, H), e(2 * O)
    p1, p1b, p2, p2b = e(Q, 2 * Q), e(Q), e(2, Q), e(2)
    outs = [(w12, None), (u1, u1b), (u2, u2b), (v12, None), (p1, p1b), (p2, p2b)]
    ops = _head_factor_ops(n, H, *factors)
    probs = [{"A": A, "B": B, "C": C} if Cb is None else {"A": A, "B": B, "C": C, "Cb": Cb}
             for (A, B), (C, Cb) in zip(ops, outs)]
    if seg2 is not None:
        for p, (A2, B2) in zip(probs, _head_factor_ops(seg2[0], H, *seg2[1])):
            p.update(A2=A2, B2=B2)
    wgrad_tn(probs)
    return [w12[:H], w12[H:], u1, u1b, u2, u2b, v12[:Q], v12[Q:], p1, p1b, p2, p2b]


def _eq_head_weight_grads(lib, x, vec, params, gy, gx, gv, seg2=None, stash=None):
    """tmdnet_eq_head_bwd_weights (g_x, g_vec and the per-atom factors) + one GEMM per weight pair
    (``seg2``: the HVP's factor rows, summed by the same GEMMs; ``stash``: a _HeadLink to leave this
    pass's factor rows at instead -- returns None)."""
    N, H = x.shape
    O = Q = H // 2
    o = dict(dtype=x.dtype, device=x.device)
    a1 = torch.empty((N, 3, H + O), **o)
    gu = torch.empty((N, H), **o)
    hext = torch.empty((N, 2 * H + 1), **o)
    go = torch.empty((N, 2 * O), **o)
    sext = torch.empty((N, H + 1), **o)
    a2 = torch.empty((N, 3, Q + 1), **o)
    v1 = torch.empty((N, 3, O), **o)
    gu2 = torch.empty((N, Q), **o)
    h2ext = torch.empty((N, 2 * Q + 1), **o)
    go2 = torch.empty((N, 2), **o)
    s2ext = torch.empty((N, Q + 1), **o)
    saves = [a1, gu, hext, go, sext, a2, v1, gu2, h2ext, go2, s2ext]
    ws = (ctypes.c_void_p * 12)(*[p.data_ptr() for p in params])
    sv = (ctypes.c_void_p * 11)(*[t.data_ptr() for t in saves])
    rc = lib.tmdnet_eq_head_bwd_weights(nat.dtype_code(x.dtype), N, H, nat.ptr(x), nat.ptr(vec), ws,
                                        nat.ptr(gy), nat.ptr(gx), nat.ptr(gv), sv, nat.stream(x.device))
    nat.check(rc, "tmdnet_eq_head_bwd_weights")
    if stash is not None:
        stash.leave("fwd", (N, (a1, vec, gu, hext, go, sext, a2, v1, gu2, h2ext, go2, s2ext)))
        return None
    return _head_wgrads(N, H, a1, vec, gu, hext, go, sext, a2, v1, gu2, h2ext, go2, s2ext, seg2=seg2)


class _EqHeadBwd(Function):
    """First-order backward of the head: g_x, g_vec = g_y * Jacobian (HIP); the weight gradients
    (training only) and every second-order term come from the composite."""

    @staticmethod
    def forward(ctx, opts, gy, jx, jv, x, vec, *params):
        need_w, seg2, stash = opts
        lib = nat.load()
        N, H = x.shape
        gx = torch.empty_like(x)
        gv = torch.empty_like(vec)
        g_params = [None] * len(params)
        if need_w:
            g_params = _eq_head_weight_grads(lib, x, vec, params, gy, gx, gv, seg2=seg2, stash=stash)
            g_params = [None] * len(params) if g_params is None else g_params
        else:
            if jx is None:
                raise RuntimeError("torchmd-net_amd: head Jacobian was not computed in the forward")
            rc = lib.tmdnet_eq_head_bwd(nat.dtype_code(x.dtype), N, H, nat.ptr(gy), nat.ptr(jx), nat.ptr(jv),
                                        nat.ptr(gx), nat.ptr(gv), nat.stream(x.device))
            nat.check(rc, "tmdnet_eq_head_bwd")
        ctx.set_materialize_grads(False)  # unused outputs (the weight gradients) stay None
        ctx.save_for_backward(gy, x, vec, *params)
        return (gx, gv) + tuple(g_params)

    @staticmethod
    def backward(ctx, ggx, ggv, *ggp):
        saved = ctx.saved_tensors
        _create = torch.is_grad_enabled()  # third order only if the caller builds a graph
        if not _create and all(g is None for g in ggp) and HEAD_SECOND_ORDER != "composite":
            gy, x, vec, *params = saved
            need_p = [ctx.needs_input_grad[6 + i] for i in range(len(params))]
            # the head's forward node also computes weight gradients in this pass (the energy loss): one
            # grouped GEMM for both (_HeadLink)
            link = getattr(ctx, "link", None) if (any(need_p) and HEAD_HANDOFF) else None
            seg2 = link.take("hvp") if link is not None else None
            hand = link is not None and seg2 is None and link.other_will_run("hvp")
            d_gy, d_x, d_vec, d_p = eq_head_hvp(x, vec, params, gy, ggx, ggv, ctx.needs_input_grad[1], any(need_p),
                                                factors_only=hand, seg2=seg2)
            if hand:
                link.leave("hvp", d_p)
                d_p = None
            d_p = [g if w else None for g, w in zip(d_p, need_p)] if d_p is not None else [None] * len(params)
            return (None, d_gy, None, None, d_x, d_vec) + tuple(d_p)
        with torch.enable_grad():
            leaves = [t.detach().requires_grad_(True) for t in saved]
            gy, x, vec = leaves[:3]
            ps = leaves[3:]
            y = eq_head_composite(x, vec, ps)
            first = torch.autograd.grad(y, [x, vec] + ps, gy, create_graph=True, allow_unused=True)
            sel = [(f, g) for f, g in zip(first, (ggx, ggv) + tuple(ggp)) if f is not None and g is not None]
            if not sel:
                return (None,) * (6 + len(ps))
            second = torch.autograd.grad([f for f, _ in sel], leaves, [g for _, g in sel],
                                         create_graph=_create, allow_unused=True)
        d_gy, d_x, d_vec = second[:3]
        return (None, d_gy, None, None, d_x, d_vec) + tuple(second[3:])


def eq_head_hvp(x, vec, params, gy, tx, tv, want_gy=True, want_w=True, factors_only=False, seg2=None):
    """Second order of the head's backward (tmdnet_eq_head_hvp, forward-over-reverse in one kernel):
    returns (d_gy [N,1] or None, d_x, d_vec, [12 weight terms] or None) for the cotangents (tx, tv)
    of (g_x, g_vec) = gy * J(x, vec); each weight term is one GEMM over the kernel's per-atom
    factors ([tangent rows ; plain rows], the layouts of _eq_head_weight_grads).  ``factors_only``:
    the fourth item is (2N, factor rows) for _head_wgrads' seg2 instead of the weight terms; ``seg2``:
    the first-order pass's factor rows, summed by the same GEMMs."""
    lib = nat.load()
    N, H = x.shape
    O = Q = H // 2
    o = dict(dtype=x.dtype, device=x.device)
    d_x = torch.empty_like(x)
    d_vec = torch.empty_like(vec)
    d_gy = torch.empty((N, 1), **o) if want_gy else None
    tx = None if tx is None else tx.contiguous()
    tv = None if tv is None else tv.contiguous()
    saves = None
    sv = None
    if want_w:
        n2 = 2 * N
        saves = [torch.empty((n2, 3, H + O), **o), torch.empty((n2, H), **o), torch.empty((n2, 2 * H + 1), **o),
                 torch.empty((n2, 2 * O), **o), torch.empty((n2, H + 1), **o), torch.empty((n2, 3, Q + 1), **o),
                 torch.empty((n2, 3, O), **o), torch.empty((n2, Q), **o), torch.empty((n2, 2 * Q + 1), **o),
                 torch.empty((n2, 2), **o), torch.empty((n2, Q + 1), **o), torch.empty((n2, 3, H), **o)]
        sv = (ctypes.c_void_p * 12)(*[t.data_ptr() for t in saves])
    ws = (ctypes.c_void_p * 12)(*[p.data_ptr() for p in params])
    rc = lib.tmdnet_eq_head_hvp(nat.dtype_code(x.dtype), N, H, nat.ptr(x), nat.ptr(vec), ws, nat.ptr(gy.contiguous()),
                                nat.ptr(tx), nat.ptr(tv), nat.ptr(d_x), nat.ptr(d_vec), nat.ptr(d_gy), sv,
                                nat.stream(x.device))
    nat.check(rc, "tmdnet_eq_head_hvp")
    if saves is None:
        return d_gy, d_x, d_vec, None
    a1, gu, hext, go, sext, a2, v1, gu2, h2ext, go2, s2ext, vv = saves
    if factors_only:
        return d_gy, d_x, d_vec, (2 * N, (a1, vv, gu, hext, go, sext, a2, v1, gu2, h2ext, go2, s2ext))
    d_p = _head_wgrads(2 * N, H, a1, vv, gu, hext, go, sext, a2, v1, gu2, h2ext, go2, s2ext, seg2=seg2)
    return d_gy, d_x, d_vec, d_p


def eq_scalar_head(x, vec, blocks):
    """EquivariantScalar.pre_reduce's two gated blocks through the fused HIP head."""
    nat.require_gpu(x, "eq_scalar_head")
    return _EqHead.apply(x, vec, *eq_head_params(blocks))


# ----------------------------------------------------------------------------- embeddings and Linears
# with hand-written weight gradients.  The library GEMM picks few-workgroup tiles with a serial K loop
# for the "sum over rows" weight gradients of the neighbour embedding's Linears (e.g. 112 us for
# [128 x 12548] [12548 x 64] at ET-QM9) and embedding_dense_backward sorts the indices (48 us per
# table): both are TN GEMMs here (tmdnet_gemm_tn_f32 / tmdnet_embedding_bwd_f32), deterministic.
def _tn_ok(*ts):
    return all(t is None or (t.is_cuda and t.dtype == torch.float32) for t in ts)


def embedding_fwd(z, weights):
    """weights[t][z] for every table (rows of H fp32): one tmdnet_embedding_fwd_f32 launch on the GPU
    (the two lookups of TorchMD_ET / NeighborEmbedding); ``index_select`` for fp64 / CPU tensors."""
    H = weights[0].shape[1]
    if (not _tn_ok(*weights) or H % 4 or len(weights) > 4 or any(w.shape[1] != H for w in weights)
            or any(w.stride(1) != 1 or w.stride(0) % 4 or w.data_ptr() % 16 for w in weights)):
        return tuple(w.index_select(0, z) for w in weights)
    outs = [torch.empty((z.shape[0], H), dtype=w.dtype, device=w.device) for w in weights]
    n = len(weights)
    tp = (ctypes.c_void_p * n)(*[w.data_ptr() for w in weights])
    lt = (ctypes.c_int * n)(*[w.stride(0) for w in weights])
    op = (ctypes.c_void_p * n)(*[o.data_ptr() for o in outs])
    zc = z.to(torch.int64).contiguous()
    rc = nat.load().tmdnet_embedding_fwd_f32(z.shape[0], H, weights[0].shape[0], nat.ptr(zc), n, tp, lt, op,
                                             None, nat.stream(z.device))
    nat.check(rc, "tmdnet_embedding_fwd_f32")
    return tuple(outs)


def embedding_bwd(z, grads, num_types, out=None, accumulate=False):
    """Table gradients of embeddings looked up at ``z``: one launch for every (grad [n, H]) of ``grads``."""
    H = grads[0].shape[1]
    outs = out if out is not None else [torch.empty((num_types, H), dtype=g.dtype, device=g.device) for g in grads]
    if not _tn_ok(*grads):
        for g, o in zip(grads, outs):
            if not accumulate:
                o.zero_()
            o.index_add_(0, z, g)
        return outs
    gs = [g if g.stride(1) == 1 else g.contiguous() for g in grads]
    n = len(gs)
    gp = (ctypes.c_void_p * n)(*[g.data_ptr() for g in gs])
    ld = (ctypes.c_int * n)(*[g.stride(0) for g in gs])
    op = (ctypes.c_void_p * n)(*[o.data_ptr() for o in outs])
    rc = nat.load().tmdnet_embedding_bwd_f32(z.shape[0], H, num_types, nat.ptr(z), n, gp, ld, op,
                                             int(bool(accumulate)), nat.stream(z.device))
    nat.check(rc, "tmdnet_embedding_bwd_f32")
    return outs


class _Embedding(Function):
    """weights[t][z] for every table t (reference nn.Embedding; TorchMD_ET's and NeighborEmbedding's
    tables share z): both lookups one node, both table gradients one launch."""

    @staticmethod
    def forward(ctx, z, *weights):
        ctx.save_for_backward(z)
        ctx.shapes = [w.shape for w in weights]
        return embedding_fwd(z, weights)

    @staticmethod
    def backward(ctx, *gs):
        z, = ctx.saved_tensors
        live = [i for i, g in enumerate(gs) if g is not None and ctx.needs_input_grad[1 + i]]
        res = [None] * len(gs)
        if live:
            if torch.is_grad_enabled():  # a graph of this gradient (third order): differentiable composite
                for i in live:
                    res[i] = torch.zeros(ctx.shapes[i], dtype=gs[i].dtype, device=gs[i].device).index_add(0, z, gs[i])
            else:
                outs = embedding_bwd(z, [gs[i] for i in live], ctx.shapes[live[0]][0])
                for i, o in zip(live, outs):
                    res[i] = o
        return (None,) + tuple(res)


def embedding(z, *weights):
    return _Embedding.apply(z, *weights)


class _Linear(Function):
    """y = x W^T + b (reference nn.Linear) whose backward forms only the gradients the engine will
    consume; its weight / bias gradient is one TN launch (bias = the ones column)."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_b = b is not None
        if x.dim() == 2 and x.is_cuda and x.dtype == torch.float32:  # hand-written MFMA GEMM (tmdnet_gemm_f32)
            y = torch.empty((x.shape[0], w.shape[0]), dtype=x.dtype, device=x.device)
            if gemm_launch([(x, w, True, b, y, False)]):
                return y
            if x.shape[0] > GEMM_MAX_ROWS and gemm_x3(x, w, True, b, y, False):
                return y
        return F.linear(x, w, b)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        nf = ctx.next_functions
        need = (ctx.needs_input_grad[0] and _will_run(nf[0][0]),
                ctx.needs_input_grad[1] and _will_run(nf[1][0]),
                ctx.has_b and ctx.needs_input_grad[2] and _will_run(nf[2][0]))
        if not any(need):
            return None, None, None
        gx, gw, gb = _LinearBwd.apply(gy, x, w, need)
        return gx, gw, gb


def _linear_wgrad(gy, x, want_w, want_b, seg2=None, rows=None):
    """(g_W, g_b) = (gy^T x, sum gy) [+ seg2 = (gy2, x2): gy2^T x2] in one TN launch (fp32 CUDA); ``rows``
    (int32 device scalar): only the first rows of each segment are non-zero (see wgrad_tn)."""
    out_f, in_f = gy.shape[1], x.shape[1]
    if not _tn_ok(gy, x) or gy.stride(1) != 1 or x.stride(1) != 1:
        gw = (gy.t() @ x + (seg2[0].t() @ seg2[1] if seg2 is not None else 0)) if want_w else None
        return gw, (gy.sum(0) if want_b else None)
    o = dict(dtype=gy.dtype, device=gy.device)
    gw = torch.empty((out_f, in_f), **o) if want_w else None
    gb = torch.empty((out_f,), **o) if want_b else None
    if want_w:  # the bias (ones column) lands in its own contiguous vector
        p = {"A": gy, "B": x, "C": gw, "Cb": gb, "ones": bool(want_b)}
        if seg2 is not None:
            p.update(A2=seg2[0], B2=seg2[1], ones2=False)
    else:
        p = {"A": gy, "B": None, "C": gb.view(out_f, 1), "ones": True}
    if rows is not None:
        p["rows"] = rows
    wgrad_tn([p])
    return gw, gb


class _LinearBwd(Function):
    """(gx, gW, gb) of _Linear, itself differentiable (force-matching training differentiates the
    force pass): for cotangents (ggx, ggW, ggb),  d gy = ggx W + x ggW^T + ggb,  d x = gy ggW,
    d W = gy^T ggx."""

    @staticmethod
    def forward(ctx, gy, x, w, need):
        gx = None
        if need[0]:
            gy = gy.contiguous()
            gx = torch.empty((gy.shape[0], w.shape[1]), dtype=gy.dtype, device=gy.device)
            if not (gy.is_cuda and (gemm_launch([(gy, w, False, None, gx, False)])
                                    or (gy.shape[0] > GEMM_MAX_ROWS and gemm_x3(gy, w, False, None, gx, False)))):
                torch.mm(gy, w, out=gx)
        gw, gb = _linear_wgrad(gy, x, need[1], need[2]) if (need[1] or need[2]) else (None, None)
        ctx.save_for_backward(gy, x, w)
        return gx, gw, gb

    @staticmethod
    def backward(ctx, ggx, ggw, ggb):
        gy, x, w = ctx.saved_tensors
        nf = ctx.next_functions
        want = [ctx.needs_input_grad[i] and _will_run(nf[i][0]) for i in range(3)]
        d_gy = d_x = d_w = None
        hand = gy.is_cuda and gy.dtype == torch.float32 and not torch.is_grad_enabled()
        if want[0] and hand and (ggx is not None or ggw is not None):
            # d gy = ggx W + x ggW^T + ggb on the hand GEMMs (the bias on the first, the second accumulating)
            d_gy = torch.empty_like(gy)
            probs = []
            if ggx is not None:
                probs.append((ggx.contiguous(), w, True, ggb, d_gy, False))
            if ggw is not None:
                probs.append((x.contiguous(), ggw.contiguous(), True, ggb if not probs else None, d_gy, bool(probs)))
            for q in probs:
                gemm_group([q])
        elif want[0]:
            parts = []
            if ggx is not None:
                parts.append(ggx @ w.t())
            if ggw is not None:
                parts.append(x @ ggw.t())
            if ggb is not None:
                parts.append(ggb.expand(gy.shape))
            if parts:
                d_gy = parts[0]
                for t in parts[1:]:
                    d_gy = d_gy + t
        if want[1] and ggw is not None:
            if hand:
                d_x = torch.empty((gy.shape[0], ggw.shape[1]), dtype=gy.dtype, device=gy.device)
                gemm_group([(gy.contiguous(), ggw.contiguous(), False, None, d_x, False)])
            else:
                d_x = gy @ ggw
        if want[2] and ggx is not None:
            if torch.is_grad_enabled():
                d_w = gy.t() @ ggx
            else:
                d_w, _ = _linear_wgrad(gy, ggx, True, False)
        return d_gy, d_x, d_w, None


def linear(x, w, b=None):
    return _Linear.apply(x, w, b)


# ----------------------------------------------------------------------------- Linear + SiLU stacks
def gemm_ex_launch(problems):
    """``tmdnet_gemm_ex_f32``: up to 4 problems, dicts with A, B, C and optional trans_b (default True),
    bias, beta, act (0/1), pre, rscale, dpre (pre / dpre share a row stride).  Returns False when
    outside the kernel's envelope (nothing launched)."""
    if not problems or len(problems) > 4:
        return False
    if any(p["A"].shape[0] > GEMM_MAX_ROWS for p in problems):
        # large systems: one tmdnet_gemm_x3_ex_f32 launch per problem (same epilogue), all or nothing
        ok = [_x3_ex_ok(p) for p in problems]
        if not all(ok):
            return False
        for p in problems:
            if not gemm_x3(p["A"], p["B"], p.get("trans_b", True), p.get("bias"), p["C"], p.get("beta"),
                           act=int(p.get("act", 0)), pre=p.get("pre"), rscale=p.get("rscale"), dpre=p.get("dpre")):
                raise RuntimeError("gemm_ex_launch: tmdnet_gemm_x3_ex_f32 refused a checked problem")
        return True
    for p in problems:
        A, C = p["A"], p["C"]
        if (A.dtype != torch.float32 or not A.is_cuda or not 0 < A.shape[0] <= GEMM_MAX_ROWS or A.shape[1] == 0
                or C.shape[1] == 0 or A.stride(1) != 1 or p["B"].stride(1) != 1 or C.stride(1) != 1):
            return False
    lib = nat.load()
    n = len(problems)
    dims = (ctypes.c_int * (10 * n))()
    ptrs = (ctypes.c_void_p * (7 * n))()
    for i, p in enumerate(problems):
        A, B, C = p["A"], p["B"], p["C"]
        x = p.get("pre") if p.get("pre") is not None else p.get("dpre")
        if x is not None and (x.stride(1) != 1 or x.shape != C.shape):
            return False
        dims[10 * i:10 * i + 10] = [A.shape[0], C.shape[1], A.shape[1], A.stride(0), B.stride(0), C.stride(0),
                                    int(p.get("trans_b", True)), int(bool(p.get("beta"))), int(p.get("act", 0)),
                                    0 if x is None else x.stride(0)]
        ptrs[7 * i:7 * i + 7] = [A.data_ptr(), B.data_ptr()] + [
            None if p.get(k) is None else p[k].data_ptr() for k in ("bias", "C", "pre", "rscale", "dpre")]
    rc = lib.tmdnet_gemm_ex_f32(n, dims, ptrs, nat.stream(problems[0]["A"].device))
    if rc == GEMM_UNSUPPORTED:
        return False
    nat.check(rc, "tmdnet_gemm_ex_f32")
    return True


def _x3_ex_ok(p):
    """Whether gemm_x3 takes problem p (the x3 kernel's envelope, checked before anything launches)."""
    A, B, C = p["A"], p["B"], p["C"]
    bias, x = p.get("bias"), (p.get("pre") if p.get("pre") is not None else p.get("dpre"))
    return (GEMM_BIG == "x3" and A.is_cuda and all(t.dtype == torch.float32 for t in (A, B, C))
            and A.shape[0] > 0 and A.shape[1] % 32 == 0 and C.shape[1] % 16 == 0
            and A.stride(1) == 1 and B.stride(1) == 1 and C.stride(1) == 1
            and A.stride(0) % 4 == 0 and B.stride(0) % 4 == 0 and C.stride(0) % 4 == 0
            and (bias is None or bias.is_contiguous()) and _al16(A, B, C, bias, p.get("pre"), p.get("dpre"))
            and (x is None or (x.stride(1) == 1 and x.stride(0) % 4 == 0 and x.shape == C.shape)))


def _mlp_composite(x, scale, *wb):
    """Differentiable restatement: silu(Linear) layers, the last one times scale[:, None]."""
    L = len(wb) // 2
    h = x
    for i in range(L):
        h = F.silu(F.linear(h, wb[i], wb[L + i]))
    return h if scale is None else h * scale.view(-1, 1)


class _MLPAct(Function):
    """h_{i+1} = silu(h_i W_i^T + b_i), the last layer times a per-row scale (reference tensornet.py
    edge MLP 381-385 with the cutoff, embedding MLP 320-321, output head 233): every layer ONE
    tmdnet_gemm_ex_f32 launch with the activation (and the pre-activation a backward needs) in its
    epilogue -- the separate activation launch per layer is gone.  The backward runs the chain with
    each layer's silu' in the epilogue of the GEMM that produces the gradient feeding it, and all
    weight / bias gradients in one grouped TN launch."""

    @staticmethod
    def forward(ctx, x, scale, *wb):
        L = len(wb) // 2
        ws, bs = wb[:L], wb[L:]
        o = dict(dtype=x.dtype, device=x.device)
        h, pres, hs = x, [], []
        for i in range(L):
            pre = torch.empty((x.shape[0], ws[i].shape[0]), **o)
            y = torch.empty_like(pre)
            ok = gemm_ex_launch([{"A": h, "B": ws[i], "bias": bs[i], "C": y, "pre": pre, "act": 1,
                                  "rscale": scale if i == L - 1 else None}])
            if not ok:
                raise RuntimeError("mlp_act: shape outside tmdnet_gemm_ex_f32's envelope")
            pres.append(pre)
            hs.append(h)
            h = y
        ctx.L = L
        ctx.save_for_backward(x, scale, *ws, *bs, *pres, *hs[1:])
        return h

    @staticmethod
    def backward(ctx, gy):
        L = ctx.L
        sv = ctx.saved_tensors
        x, scale = sv[0], sv[1]
        ws, bs = sv[2:2 + L], sv[2 + L:2 + 2 * L]
        pres, hmid = sv[2 + 2 * L:2 + 3 * L], sv[2 + 3 * L:]
        # next_functions has no entry for a None input (scale may be None): index by tensor inputs
        nf = ctx.next_functions
        at = [i - (1 if (scale is None and i > 1) else 0) for i in range(2 + 2 * L)]
        need = [ctx.needs_input_grad[i] and _will_run(nf[at[i]][0]) for i in range(2 + 2 * L)]
        if not any(need):
            return (None,) * (2 + 2 * L)
        outs = _MLPActBwd.apply(tuple(need), gy.contiguous(), x, scale, *ws, *bs, *pres, *hmid)
        return tuple(o if n else None for o, n in zip(outs, need))


class _MLPActBwd(Function):
    @staticmethod
    def forward(ctx, need, gy, x, scale, *rest):
        L = (len(rest) + 1) // 4
        ws, bs, pres, hmid = rest[:L], rest[L:2 * L], rest[2 * L:3 * L], rest[3 * L:]
        hs = (x,) + tuple(hmid)
        o = dict(dtype=x.dtype, device=x.device)
        # the last layer: g_pre = gy * scale * silu'(pre), g_scale = sum_c gy * silu(pre) (tmdnet_silu_bwd)
        gpre = torch.empty_like(pres[-1])
        gs = torch.empty(x.shape[0], **o) if (scale is not None and need[1]) else None
        silu_bwd_launch(pres[-1], scale, gy, gpre, gs)
        gpres = [None] * L
        gpres[L - 1] = gpre
        ups = [None] * L  # a_{i-1} = g_pre_i W_i before the silu' factor (the hand second order reads them)
        gx = None
        for i in range(L - 1, -1, -1):
            if i > 0:  # the lower layer's pre-activation gradient: (g_pre_i W_i) * silu'(pre_{i-1})
                g = torch.empty_like(pres[i - 1])
                ups[i - 1] = torch.empty_like(pres[i - 1])
                gemm_ex_launch([{"A": gpres[i], "B": ws[i], "trans_b": False, "C": g, "dpre": pres[i - 1],
                                 "pre": ups[i - 1]}]) or _raise("mlp_act backward: GEMM envelope")
                gpres[i - 1] = g
            elif need[0]:
                gx = torch.empty_like(x)
                gemm_ex_launch([{"A": gpres[0], "B": ws[0], "trans_b": False, "C": gx}]) or \
                    _raise("mlp_act backward: GEMM envelope")
        gw, gb = [None] * L, [None] * L
        tn = []
        for i in range(L):
            wn, bn = need[2 + i], need[2 + L + i]
            if wn or bn:
                gw[i] = torch.empty_like(ws[i]) if wn else None
                gb[i] = torch.empty_like(bs[i]) if bn else None
                if wn:
                    tn.append({"A": gpres[i], "B": hs[i], "C": gw[i], "Cb": gb[i], "ones": bool(bn)})
                else:
                    tn.append({"A": gpres[i], "B": None, "C": gb[i].view(-1, 1), "ones": True})
        wgrad_tn(tn)
        ctx.save_for_backward(gy, x, scale, *ws, *bs, *pres, *hmid, *gpres, *ups[:L - 1])
        ctx.L = L
        return (gx, gs, *gw, *gb)

    @staticmethod
    def backward(ctx, *ggs):
        from . import tn_node
        from .tn_node import _double_backward
        L = ctx.L
        sv = ctx.saved_tensors
        gy, x, scale = sv[0], sv[1], sv[2]
        if tn_node.SECOND_ORDER != "composite" and not torch.is_grad_enabled() and x.is_cuda \
                and x.dtype == torch.float32:
            return _mlp_second_order(ctx, sv, ggs)
        wb = list(sv[3:3 + 2 * L])
        d = _double_backward(_mlp_composite, [x, scale] + wb, [gy], list(ggs))
        # (need, gy, x, scale, *ws, *bs, *pres, *hmid): pres / hmid are functions of the others
        return (None, d[0], d[1], d[2], *d[3:3 + 2 * L]) + (None,) * (2 * L - 1)


def _raise(msg):
    raise RuntimeError(msg)


def _mlp_second_order(ctx, sv, ggs):
    """Hand-written VJP of _MLPActBwd (the Linear + SiLU stack's first backward: a_{L-1} = gy s, g_i = a_i
    silu'(p_i), a_{i-1} = g_i W_i, gW_i = g_i^T h_i, gb_i = colsum g_i, gx = g_0 W_0, gs = rowsum gy silu(p_{L-1}))
    for cotangents (X, S, Wbar_i, Bbar_i) of (gx, gs, gW_i, gb_i), instead of autograd's double differentiation
    of the composite (~100 launches per TensorNet edge MLP).  Up the layers, the adjoint of g_i,
        ghat_i = (i = 0: X W_0^T | else ahat_{i-1} W_i^T) + h_i Wbar_i^T + Bbar_i,
    gives ahat_i = ghat_i silu'(p_i) and the adjoint of p_i, dp_i = ghat_i a_i silu''(p_i) (last layer: + the gs
    terms, and the adjoints of gy and s) (tmdnet_mlp2_up); the h_i adjoints g_i Wbar_i and the W_i adjoints
    g_i^T (X | ahat_{i-1}) are injected.  Down the layers the p / h adjoints go back through the forward:
    c_i = dp_i + dh_{i+1} silu'(p_i) (tmdnet_mlp2_down), dW_i += c_i^T h_i, db_i = colsum c_i, dh_i = c_i W_i +
    g_i Wbar_i, dx = dh_0.  GEMMs on the hand-written kernels (gemm_group, wgrad_tn)."""
    L = ctx.L
    gy, x, scale = sv[0], sv[1], sv[2]
    ws, bs = sv[3:3 + L], sv[3 + L:3 + 2 * L]
    pres, hmid = sv[3 + 2 * L:3 + 3 * L], sv[3 + 3 * L:2 + 4 * L]
    gpres, ups = sv[2 + 4 * L:2 + 5 * L], sv[2 + 5 * L:]
    hs = (x,) + tuple(hmid)
    X, S = ggs[0], ggs[1]
    Wb, Bb = ggs[2:2 + L], ggs[2 + L:2 + 2 * L]
    need = ctx.needs_input_grad  # (need, gy, x, scale, *ws, *bs, *pres, *hmid)
    M = x.shape[0]
    o = dict(dtype=x.dtype, device=x.device)
    lib = nat.load()
    st = nat.stream(x.device)
    dps, ahats, injs = [None] * L, [None] * L, [None] * L
    dgy = torch.empty_like(gy) if need[1] else None
    ds = torch.empty(M, **o) if (scale is not None and need[3]) else None
    for i in range(L):
        N = ws[i].shape[0]
        ghat = torch.empty((M, N), **o)
        up = X if i == 0 else ahats[i - 1]
        probs = []
        if up is not None:
            probs.append((up.contiguous(), ws[i], True, None, ghat, False))
        if Wb[i] is not None:
            probs.append((hs[i], Wb[i].contiguous(), True, None, ghat, bool(probs)))
        if not probs:
            ghat.zero_()
        for q in probs:  # (sequential: the second accumulates)
            gemm_group([q])
        if Bb[i] is not None:
            ghat.add_(Bb[i])
        ah, dp = torch.empty_like(ghat), torch.empty_like(ghat)
        last = i == L - 1
        rc = lib.tmdnet_mlp2_up(nat.dtype_code(x.dtype), M, N, nat.ptr(pres[i]), pres[i].stride(0), nat.ptr(ghat),
                                None if last else nat.ptr(ups[i]), 0 if last else ups[i].stride(0),
                                nat.ptr(gy) if last else None, nat.ptr(scale) if last else None,
                                nat.ptr(S.contiguous()) if (last and S is not None) else None, nat.ptr(ah), nat.ptr(dp),
                                nat.ptr(dgy) if last else None, nat.ptr(ds) if last else None, st)
        nat.check(rc, "tmdnet_mlp2_up")
        ahats[i], dps[i] = ah, dp
        if Wb[i] is not None:  # gW_i = g_i^T h_i -> the adjoint of h_i gets g_i Wbar_i
            injs[i] = torch.empty_like(hs[i])
            gemm_group([(gpres[i], Wb[i].contiguous(), False, None, injs[i], False)])
    if dgy is not None and not need[1]:
        dgy = None
    dW = [torch.empty_like(w) if need[4 + i] else None for i, w in enumerate(ws)]
    dB = [torch.empty_like(b) if need[4 + L + i] else None for i, b in enumerate(bs)]
    dx = None
    c = dps[L - 1]
    for i in range(L - 1, -1, -1):
        up = X if i == 0 else ahats[i - 1]
        if dW[i] is not None or dB[i] is not None:
            prob = {"A": c, "B": hs[i] if dW[i] is not None else None,
                    "C": dW[i] if dW[i] is not None else dB[i].view(-1, 1),
                    "Cb": dB[i] if (dW[i] is not None and dB[i] is not None) else None,
                    "ones": dB[i] is not None}
            if dW[i] is not None and up is not None:  # + g_i^T (X | ahat_{i-1}) (from gx = g_0 W_0 / a_{i-1} = g_i W_i)
                prob.update(A2=gpres[i], B2=up.contiguous())
            wgrad_tn([prob])
        if i == 0 and not need[2]:
            break
        dh = torch.empty_like(hs[i])
        gemm_group([(c, ws[i], False, None, dh, False)])
        if injs[i] is not None:
            dh.add_(injs[i])
        if i == 0:
            dx = dh
        else:
            cn = torch.empty_like(dps[i - 1])
            rc = lib.tmdnet_mlp2_down(nat.dtype_code(x.dtype), M, cn.shape[1], nat.ptr(pres[i - 1]),
                                      pres[i - 1].stride(0), nat.ptr(dh), nat.ptr(dps[i - 1]), nat.ptr(cn), st)
            nat.check(rc, "tmdnet_mlp2_down")
            c = cn
    n_rest = len(ctx.needs_input_grad) - 4 - 2 * L
    return (None, dgy, dx, ds, *dW, *dB) + (None,) * n_rest


# TMDNET_MLP_ACT=0: the Linear + fused_act composite per layer instead (A/B switch)
MLP_ACT = os.environ.get("TMDNET_MLP_ACT", "1") not in ("0", "off")


def mlp_act(x, weights, biases, act, scale=None):
    """``act(... act(x W_0^T + b_0) ...) * scale[:, None]`` for nn.Linear weights / biases: the hand
    fused path for SiLU on fp32 CUDA rows within the GEMM envelope, else Linear + fused_act per layer."""
    L = len(weights)
    # (above GEMM_MAX_ROWS rows every GEMM runs on tmdnet_gemm_x3_ex_f32, which needs K % 32 in both directions)
    big = x.dim() == 2 and x.shape[0] > GEMM_MAX_ROWS
    mod = 32 if big else 16
    ok = (MLP_ACT and isinstance(act, torch.nn.SiLU) and x.is_cuda and x.dtype == torch.float32 and x.dim() == 2
          and 0 < x.shape[0] and (not big or GEMM_BIG == "x3") and all(b is not None for b in biases)
          and all(w.shape[1] % mod == 0 for w in weights) and all(w.shape[0] % mod == 0 for w in weights))
    if ok:
        # tmdnet_gemm_ex_f32 also needs 16-byte aligned operands (a contiguous view with a storage offset
        # may not be): realign x by a copy, take the composite for misaligned weights
        x = x.contiguous()
        if x.data_ptr() % 16:
            x = x.clone()
        ok = all(w.is_contiguous() and w.data_ptr() % 16 == 0 for w in weights) and \
            all(b.data_ptr() % 16 == 0 for b in biases) and (scale is None or scale.contiguous().data_ptr() % 16 == 0)
    if not ok:
        for i in range(L):
            x = fused_act(act, linear(x, weights[i], biases[i]), scale if i == L - 1 else None)
        return x
    return _MLPAct.apply(x, None if scale is None else scale.contiguous(), *weights, *biases)


# ----------------------------------------------------------------------------- LayerNorm
def _ln_composite(x, w, b, eps):
    return F.layer_norm(x, (x.shape[-1],), w, b, eps)


class _LayerNorm(Function):
    """nn.LayerNorm over the last dimension (TensorNet init_norm / out_norm, reference tensornet.py:232,
    322) on tmdnet_layernorm_fwd_f32; its backward is _LayerNormBwd (HIP first order)."""

    @staticmethod
    def forward(ctx, x, w, b, eps):
        rows, C = x.shape
        y = torch.empty_like(x)
        mean = torch.empty(rows, dtype=x.dtype, device=x.device)
        rstd = torch.empty(rows, dtype=x.dtype, device=x.device)
        rc = nat.load().tmdnet_layernorm_fwd_f32(rows, C, nat.ptr(x), x.stride(0), nat.ptr(w), nat.ptr(b), float(eps),
                                                 nat.ptr(y), C, nat.ptr(mean), nat.ptr(rstd), nat.stream(x.device))
        nat.check(rc, "tmdnet_layernorm_fwd_f32")
        ctx.save_for_backward(x, w, b, mean, rstd)
        ctx.eps = eps
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w, b, mean, rstd = ctx.saved_tensors
        nf = ctx.next_functions
        need = (ctx.needs_input_grad[0] and _will_run(nf[0][0]), ctx.needs_input_grad[1] and _will_run(nf[1][0]),
                ctx.needs_input_grad[2] and _will_run(nf[2][0]))
        if not any(need):
            return None, None, None, None
        gx, gw, gb = _LayerNormBwd.apply(gy.contiguous(), x, w, b, mean, rstd, ctx.eps, need)
        return gx, gw, gb, None


def layer_norm_wgrad(gy, x, mean, rstd):
    """(g_weight, g_bias) = (sum_rows gy * xhat, sum_rows gy) of a LayerNorm over x's rows (xhat =
    (x - mean) rstd): tmdnet_layernorm_wgrad_f32 (deterministic two-pass column sums) for fp32 CUDA rows."""
    rows, C = x.shape
    if x.is_cuda and x.dtype == torch.float32 and C <= 1024 and x.stride(1) == 1 and gy.stride(1) == 1:
        lib = nat.load()
        gw, gb = torch.empty(C, dtype=x.dtype, device=x.device), torch.empty(C, dtype=x.dtype, device=x.device)
        wsb = int(lib.tmdnet_layernorm_wgrad_workspace_bytes(rows, C))
        ws = torch.empty(max(1, wsb // 4), dtype=torch.float32, device=x.device)
        rc = lib.tmdnet_layernorm_wgrad_f32(rows, C, nat.ptr(x), x.stride(0), nat.ptr(mean.contiguous()),
                                            nat.ptr(rstd.contiguous()), nat.ptr(gy), gy.stride(0), nat.ptr(gw),
                                            nat.ptr(gb), nat.ptr(ws), wsb, nat.stream(x.device))
        nat.check(rc, "tmdnet_layernorm_wgrad_f32")
        return gw, gb
    xhat = (x - mean.reshape(rows, 1)) * rstd.reshape(rows, 1)
    return (gy * xhat).sum(0), gy.sum(0)


class _LayerNormBwd(Function):
    @staticmethod
    def forward(ctx, gy, x, w, b, mean, rstd, eps, need):
        lib = nat.load()
        rows, C = x.shape
        st = nat.stream(x.device)
        gx = gw = gb = None
        if need[0]:
            gx = torch.empty_like(x)
            rc = lib.tmdnet_layernorm_bwd_f32(rows, C, nat.ptr(x), x.stride(0), nat.ptr(w), nat.ptr(mean),
                                              nat.ptr(rstd), nat.ptr(gy), gy.stride(0), nat.ptr(gx), 0, st)
            nat.check(rc, "tmdnet_layernorm_bwd_f32")
        if need[1] or need[2]:
            gw = torch.empty_like(w) if need[1] else None
            gb = torch.empty_like(w) if need[2] else None
            wsb = int(lib.tmdnet_layernorm_wgrad_workspace_bytes(rows, C))
            ws = torch.empty(max(1, wsb // 4), dtype=torch.float32, device=x.device)
            rc = lib.tmdnet_layernorm_wgrad_f32(rows, C, nat.ptr(x), x.stride(0), nat.ptr(mean), nat.ptr(rstd),
                                                nat.ptr(gy), gy.stride(0), nat.ptr(gw), nat.ptr(gb), nat.ptr(ws), wsb, st)
            nat.check(rc, "tmdnet_layernorm_wgrad_f32")
        ctx.save_for_backward(gy, x, w, b, mean, rstd)
        ctx.eps = eps
        return gx, gw, gb

    @staticmethod
    def backward(ctx, ggx, ggw, ggb):
        gy, x, w, b, mean, rstd = ctx.saved_tensors
        eps = ctx.eps
        from . import tn_node
        if tn_node.SECOND_ORDER != "composite" and not torch.is_grad_enabled() and x.is_cuda \
                and x.dtype == torch.float32 and x.shape[1] <= 1024:
            # hand second order (tmdnet_layernorm_bwd2_f32): one pass per row + the weight's column sum
            need = ctx.needs_input_grad  # gy, x, w, b, mean, rstd, eps, need
            rows, C = x.shape
            d_gy = torch.empty_like(gy) if need[0] else None
            d_x = torch.empty_like(x) if need[1] else None
            t_row = torch.empty((rows, C), dtype=x.dtype, device=x.device) if (need[2] and ggx is not None) else None
            cont = lambda t: None if t is None else t.contiguous()  # noqa: E731
            rc = nat.load().tmdnet_layernorm_bwd2_f32(
                rows, C, nat.ptr(x), x.stride(0), nat.ptr(w), nat.ptr(mean), nat.ptr(rstd), nat.ptr(gy), gy.stride(0),
                nat.ptr(cont(ggx)), nat.ptr(cont(ggw)), nat.ptr(cont(ggb)), nat.ptr(d_gy), nat.ptr(d_x), nat.ptr(t_row),
                nat.stream(x.device))
            nat.check(rc, "tmdnet_layernorm_bwd2_f32")
            d_w = None
            if need[2]:
                d_w = (gy * t_row).sum(0) if t_row is not None else torch.zeros_like(w)
            return d_gy, d_x, d_w, None, None, None, None, None
        # composite: differentiate the composite LayerNorm twice
        d = _tn_double_backward(lambda x_, w_, b_: _ln_composite(x_, w_, b_, eps), [x, w, b], [gy], [ggx, ggw, ggb])
        return d[0], d[1], d[2], d[3], None, None, None, None


def _tn_double_backward(fwd, primals, gouts, ggs):
    from .tn_node import _double_backward
    return _double_backward(fwd, primals, gouts, ggs)


def layer_norm(x, weight, bias, eps=1e-5):
    """nn.LayerNorm(C) over [rows, C]: the HIP kernels for fp32 CUDA rows of C <= 1024, else ATen."""
    if (x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and x.shape[1] <= 1024 and x.stride(1) == 1
            and weight is not None and bias is not None and weight.dtype == torch.float32):
        return _LayerNorm.apply(x, weight, bias, float(eps))
    return _ln_composite(x, weight, bias, eps)


class _StackedRows(Function):
    """torch.cat(params, 0) when the parameters already are consecutive row blocks of ``buf``
    (et_stack._stack_views): the buffer itself, no copy kernel; the gradient splits into views."""

    @staticmethod
    def forward(ctx, buf, *params):
        ctx.rows = [p.shape[0] for p in params]
        return buf.view_as(buf)

    @staticmethod
    def backward(ctx, g):
        return (None, *torch.split(g, ctx.rows, 0))


def stacked_rows(holder, name, params):
    """cat(params, 0) without a copy: the parameters are made row blocks of one buffer once (their
    ``.data`` re-pointed, as the ET stack does) and re-stacked only if that aliasing was broken
    (``.to()``, a replaced tensor).  ``holder`` keeps the buffers (a dict)."""
    from .et_stack import _is_stacked, _stack_views
    buf = holder.get(name)
    if not _is_stacked(buf, params):
        buf = _stack_views(params)
        holder[name] = buf
    return _StackedRows.apply(buf, *params)


# ----------------------------------------------------------------------------- training loss
class _MSE2(Function):
    """w1 * mse(a1, b1) + w2 * mse(a2, b2), mean reductions (reference LNNP.step's E + F loss,
    module.py:130-179): one forward and one backward launch instead of ~14 small ATen launches on the
    captured training step's critical path.  The targets b1 / b2 take no gradient."""

    @staticmethod
    def forward(ctx, a1, b1, a2, b2, w1, w2):
        a1c, b1c, a2c, b2c = (t.contiguous() for t in (a1, b1, a2, b2))
        out = torch.empty((), dtype=a1.dtype, device=a1.device)
        rc = nat.load().tmdnet_mse2_fwd(nat.dtype_code(a1.dtype), a1c.numel(), nat.ptr(a1c), nat.ptr(b1c), float(w1),
                                        a2c.numel(), nat.ptr(a2c), nat.ptr(b2c), float(w2), nat.ptr(out),
                                        nat.stream(a1.device))
        nat.check(rc, "tmdnet_mse2_fwd")
        ctx.save_for_backward(a1c, b1c, a2c, b2c)
        ctx.w = (float(w1), float(w2))
        ctx.shapes = (a1.shape, a2.shape)
        return out

    @staticmethod
    def backward(ctx, g):
        a1, b1, a2, b2 = ctx.saved_tensors
        w1, w2 = ctx.w
        if torch.is_grad_enabled():  # a graph of the loss gradient: differentiable composite
            d1 = g * w1 * 2.0 * (a1 - b1) / a1.numel()
            d2 = g * w2 * 2.0 * (a2 - b2) / a2.numel()
            return d1.view(ctx.shapes[0]), None, d2.view(ctx.shapes[1]), None, None, None
        d1 = torch.empty_like(a1) if ctx.needs_input_grad[0] else None
        d2 = torch.empty_like(a2) if ctx.needs_input_grad[2] else None
        rc = nat.load().tmdnet_mse2_bwd(nat.dtype_code(a1.dtype), a1.numel(), nat.ptr(a1), nat.ptr(b1), w1,
                                        a2.numel(), nat.ptr(a2), nat.ptr(b2), w2, nat.ptr(g.contiguous()),
                                        nat.ptr(d1), nat.ptr(d2), nat.stream(a1.device))
        nat.check(rc, "tmdnet_mse2_bwd")
        return (None if d1 is None else d1.view(ctx.shapes[0]), None,
                None if d2 is None else d2.view(ctx.shapes[1]), None, None, None)


def mse2(a1, b1, a2, b2, w1, w2):
    """w1 * F.mse_loss(a1, b1) + w2 * F.mse_loss(a2, b2) in one launch (CUDA; shapes must match)."""
    nat.require_gpu(a1, "mse2")
    if a1.shape != b1.shape or a2.shape != b2.shape:
        raise ValueError("mse2: prediction and target shapes differ")
    for t in (b1, a2, b2):  # the kernel reads all four through a1's dtype on a1's device
        if t.dtype != a1.dtype or t.device != a1.device:
            raise ValueError("mse2: all four tensors must be on one device and of one dtype")
    return _MSE2.apply(a1, b1.detach(), a2, b2.detach(), w1, w2)
