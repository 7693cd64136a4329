"""ORACLE -- test infrastructure only.  Never imported by the product package (torchmd-net_amd/);
only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it.

A plain PyTorch-CPU restatement of the reference hot path, written from the reference math with
explicit gathers (index_select) and scatter-adds (index_add), evaluated from a state_dict:

  * neighbour list: the C restatement liboracle_nl.so (nl_oracle.c <- neighbors_cpu.cpp:24-95)
  * ExpNormalSmearing / GaussianSmearing / CosineCutoff ....... models/utils.py:272-390
  * TorchMD_ET.forward + NeighborEmbedding .................... torchmd_et.py:154-187, utils.py:73-108
  * EquivariantMultiHeadAttention.forward/message/aggregate ... torchmd_et.py:272-347
  * TensorNet / TensorEmbedding / Interaction ................. tensornet.py:16-67, 200-410
  * EquivariantScalar / GatedEquivariantBlock / Scalar ........ output_modules.py:49-115, utils.py:456-522
  * TorchMD_Net.forward (sum reduce, forces = -dy/dpos) ........ model.py:232-300

Parity of this restatement is pinned against fixtures produced by running the reference itself
(tests/golden/*.npz, generator tests/golden/gen_reference_fixtures.py) -- see tests/test_oracle.py.
It is also the CPU baseline that bench.py times (``cpu_baseline.kind = "port"``).
"""
import ctypes
import math
import os

import numpy as np
import torch
import torch.nn.functional as F

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle_nl.so")
        if not os.path.exists(path):
            import subprocess
            subprocess.check_call(["make", "-C", _HERE, "liboracle_nl.so"], stdout=subprocess.DEVNULL)
        lib = ctypes.CDLL(path)
        lib.oracle_neighbors.restype = ctypes.c_long
        P = ctypes.c_void_p
        lib.oracle_neighbors.argtypes = [P, P, ctypes.c_long, P, ctypes.c_int, ctypes.c_double,
                                         ctypes.c_double, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_long, P, P, P, P]
        _LIB = lib
    return _LIB


def neighbors(pos, batch, cutoff_lower, cutoff_upper, loop=False, include_transpose=True, box=None,
              sq_compare=False):
    """Reference CPU neighbour op restated in C.  Returns numpy (nb [2,P] int64, deltas [P,3] f64,
    distances [P] f64) in the reference CPU order."""
    pos = np.ascontiguousarray(np.asarray(pos, dtype=np.float64))
    batch = np.ascontiguousarray(np.asarray(batch, dtype=np.int64))
    n = pos.shape[0]
    periodic = box is not None and np.asarray(box).size == 9
    boxa = np.ascontiguousarray(np.asarray(box, dtype=np.float64).reshape(9)) if periodic else np.zeros(9)
    lib = _lib()
    args = lambda cap, a, b, c, d: lib.oracle_neighbors(
        pos.ctypes.data, batch.ctypes.data, n, boxa.ctypes.data, int(periodic), float(cutoff_lower),
        float(cutoff_upper), int(loop), int(include_transpose), int(sq_compare), cap,
        a.ctypes.data if a is not None else None, b.ctypes.data if b is not None else None,
        c.ctypes.data if c is not None else None, d.ctypes.data if d is not None else None)
    # size query then fill
    cap = 1 << 16
    while True:
        nb0 = np.empty(cap, np.int32)
        nb1 = np.empty(cap, np.int32)
        dl = np.empty((cap, 3), np.float64)
        ds = np.empty(cap, np.float64)
        p = args(cap, nb0, nb1, dl, ds)
        if p <= cap:
            break
        cap = int(p)
    nb = np.stack([nb0[:p], nb1[:p]]).astype(np.int64)
    return nb, dl[:p], ds[:p]


def sort_pairs(nb, *per_edge):
    order = np.lexsort(nb)
    return (nb[:, order],) + tuple(a[order] for a in per_edge)


# ----------------------------------------------------------------------------- basis / cutoff
def cosine_cutoff(r, cl, cu):
    if cl > 0:
        c = 0.5 * (torch.cos(math.pi * (2 * (r - cl) / (cu - cl) + 1.0)) + 1.0)
        return c * (r < cu) * (r > cl)
    return 0.5 * (torch.cos(r * math.pi / cu) + 1.0) * (r < cu)


def expnorm(r, means, betas, cl, cu):
    alpha = 5.0 / (cu - cl)
    r = r.unsqueeze(-1)
    return cosine_cutoff(r, 0.0, cu) * torch.exp(-betas * (torch.exp(alpha * (-r + cl)) - means) ** 2)


def gauss(r, offset, coeff):
    return torch.exp(coeff * (r.unsqueeze(-1) - offset) ** 2)


def linear(sd, name, x):
    w = sd[name + ".weight"]
    b = sd.get(name + ".bias")
    return F.linear(x, w, b)


def layer_norm(sd, name, x):
    return F.layer_norm(x, (x.shape[-1],), sd[name + ".weight"], sd[name + ".bias"], 1e-5)


# ----------------------------------------------------------------------------- graph
def edge_geometry(pos, batch, cl, cu, max_pairs=None, loop=True, pad_static=False, box=None):
    """Edges (src=nb[0], dst=nb[1]) + differentiable deltas / distances (self loops: constant 0, as
    the reference CPU op appends them without a norm).  ``pad_static`` emulates the CUDA op's
    (-1,-1) padding up to ``max_pairs`` remapped to (0,0) edges by TensorNet (tensornet.py:215-221).
    ``box`` (3x3, reduced form): periodic minimum-image deltas (neighbors_cpu.cpp:69-78), carried as
    the constant image shift added to the differentiable pos[src] - pos[dst]."""
    nb, ref_dl, _ = neighbors(pos.detach().cpu().numpy(), batch.cpu().numpy(), cl, cu, loop=loop,
                              include_transpose=True, box=box)
    src = torch.as_tensor(nb[0])
    dst = torch.as_tensor(nb[1])
    shift = None
    if box is not None:
        raw = (pos.detach().index_select(0, src) - pos.detach().index_select(0, dst)).double()
        shift = (torch.as_tensor(ref_dl) - raw).to(pos.dtype)
    if pad_static:
        npad = int(max_pairs) - src.numel()
        assert npad >= 0, "fixture overflowed capacity"
        src = torch.cat([src, torch.zeros(npad, dtype=src.dtype)])
        dst = torch.cat([dst, torch.zeros(npad, dtype=dst.dtype)])
        if shift is not None:
            shift = torch.cat([shift, torch.zeros(npad, 3, dtype=shift.dtype)])
    self_edge = src == dst
    dl = pos.index_select(0, src) - pos.index_select(0, dst)
    if shift is not None:
        dl = dl + shift
    dl = torch.where(self_edge.unsqueeze(1), torch.zeros_like(dl), dl)
    sq = (dl * dl).sum(1)
    r = torch.where(self_edge, torch.zeros_like(sq), torch.where(self_edge, torch.ones_like(sq), sq).sqrt())
    return src, dst, dl, r, self_edge


# ----------------------------------------------------------------------------- ET
# the reference act_class_mapping (models/utils.py:579-584); ShiftedSoftplus subtracts log 2 rounded to
# fp32 (utils.py:354-359: torch.log(torch.tensor(2.0)).item())
SSP_SHIFT = 0.693147182464599609375
ACTS = {"silu": F.silu, "tanh": torch.tanh, "sigmoid": torch.sigmoid,
        "ssp": lambda x: F.softplus(x) - SSP_SHIFT}


def et_representation(sd, cfg, z, pos, batch, prefix="representation_model.", hooks=None):
    p = lambda n: prefix + n
    H, heads = cfg["embedding_dimension"], cfg["num_heads"]
    d = H // heads
    cl, cu = cfg["cutoff_lower"], cfg["cutoff_upper"]
    N = z.shape[0]
    x = sd[p("embedding.weight")][z]
    src, dst, dl, r, self_edge = edge_geometry(pos, batch, cl, cu, box=cfg.get("box"))
    if cfg.get("rbf_type", "expnorm") == "expnorm":
        f = expnorm(r, sd[p("distance_expansion.means")], sd[p("distance_expansion.betas")], cl, cu)
    else:
        f = gauss(r, sd[p("distance_expansion.offset")], sd[p("distance_expansion.coeff")])
    sq = (dl * dl).sum(1)
    nrm = torch.where(self_edge, torch.ones_like(sq), sq).sqrt().unsqueeze(1)
    u = torch.where(self_edge.unsqueeze(1), dl, dl / nrm)
    C = cosine_cutoff(r, cl, cu)
    if cfg.get("neighbor_embedding", True):
        keep = ~self_edge
        s_, t_, C_, f_ = src[keep], dst[keep], C[keep], f[keep]
        W = linear(sd, p("neighbor_embedding.distance_proj"), f_) * C_.unsqueeze(1)
        xn = sd[p("neighbor_embedding.embedding.weight")][z]
        agg = torch.zeros_like(x).index_add(0, t_, xn.index_select(0, s_) * W)
        x = linear(sd, p("neighbor_embedding.combine"), torch.cat([x, agg], dim=1))
    vec = torch.zeros(N, 3, H, dtype=x.dtype)
    di = cfg.get("distance_influence", "both")
    act, attn_act = ACTS[cfg.get("activation", "silu")], ACTS[cfg.get("attn_activation", "silu")]
    for li in range(cfg["num_layers"]):
        lp = p(f"attention_layers.{li}.")
        xn_ = layer_norm(sd, lp + "layernorm", x)
        q = linear(sd, lp + "q_proj", xn_).view(N, heads, d)
        k = linear(sd, lp + "k_proj", xn_).view(N, heads, d)
        v = linear(sd, lp + "v_proj", xn_).view(N, heads, 3 * d)
        vec1, vec2, vec3 = torch.split(linear(sd, lp + "vec_proj", vec), H, dim=-1)
        vec_dot = (vec1 * vec2).sum(dim=1)
        att = q.index_select(0, dst) * k.index_select(0, src)
        if di in ("keys", "both"):
            att = att * act(linear(sd, lp + "dk_proj", f)).view(-1, heads, d)
        att = attn_act(att.sum(-1)) * C.unsqueeze(1)
        vj = v.index_select(0, src)
        if di in ("values", "both"):
            vj = vj * act(linear(sd, lp + "dv_proj", f)).view(-1, heads, 3 * d)
        xm, v1, v2 = torch.split(vj, d, dim=2)
        xm = xm * att.unsqueeze(2)
        vm = vec.view(N, 3, heads, d).index_select(0, src) * v1.unsqueeze(1) + v2.unsqueeze(1) * u.view(-1, 3, 1, 1)
        xa = torch.zeros(N, heads, d, dtype=x.dtype).index_add(0, dst, xm).view(N, H)
        va = torch.zeros(N, 3, heads, d, dtype=x.dtype).index_add(0, dst, vm).view(N, 3, H)
        o1, o2, o3 = torch.split(linear(sd, lp + "o_proj", xa), H, dim=1)
        dx = vec_dot * o2 + o3
        dvec = vec3 * o1.unsqueeze(1) + va
        if hooks is not None:
            hooks[f"layer{li}/dx"] = dx
            hooks[f"layer{li}/dvec"] = dvec
        x = x + dx
        vec = vec + dvec
    x = layer_norm(sd, p("out_norm"), x)
    return x, vec


def gated_block(sd, name, x, v, out_channels, scalar_act, act=F.silu):
    vb = linear(sd, name + ".vec1_proj", v)
    nz = (vb != 0).flatten(1).any(dim=1, keepdim=True)
    sq = (vb * vb).sum(dim=-2)
    vec1 = torch.where(nz, torch.where(nz, sq, torch.ones_like(sq)).sqrt(), torch.zeros_like(sq))
    vec2 = linear(sd, name + ".vec2_proj", v)
    h = torch.cat([x, vec1], dim=-1)
    h = linear(sd, name + ".update_net.2", act(linear(sd, name + ".update_net.0", h)))
    x, v = torch.split(h, out_channels, dim=-1)
    v = v.unsqueeze(1) * vec2
    if scalar_act:
        x = act(x)
    return x, v


def equivariant_scalar(sd, cfg, x, v, prefix="output_model."):
    H = cfg["embedding_dimension"]
    act = ACTS[cfg.get("activation", "silu")]  # the head's activation is the model's (reference model.py:63-68)
    x, v = gated_block(sd, prefix + "output_network.0", x, v, H // 2, True, act)
    x, v = gated_block(sd, prefix + "output_network.1", x, v, 1, False, act)
    return x + v.sum() * 0


def scalar_head(sd, x, prefix="output_model."):
    return linear(sd, prefix + "output_network.2", F.silu(linear(sd, prefix + "output_network.0", x)))


# ----------------------------------------------------------------------------- TensorNet
def _skew(v):
    z = torch.zeros_like(v[:, 0])
    return torch.stack((z, -v[:, 2], v[:, 1], v[:, 2], z, -v[:, 0], -v[:, 1], v[:, 0], z), dim=1).view(-1, 3, 3)


def _sym(v):
    t = v.unsqueeze(-1) * v.unsqueeze(-2)
    eye = torch.eye(3, dtype=v.dtype)
    i = t.diagonal(dim1=-2, dim2=-1).mean(-1)[..., None, None] * eye
    return 0.5 * (t + t.transpose(-2, -1)) - i


def _decompose(t):
    eye = torch.eye(3, dtype=t.dtype)
    i = t.diagonal(dim1=-2, dim2=-1).mean(-1)[..., None, None] * eye
    a = 0.5 * (t - t.transpose(-2, -1))
    s = 0.5 * (t + t.transpose(-2, -1)) - i
    return i, a, s


def _tnorm(t):
    return (t ** 2).sum((-2, -1))


def _chan_linear(sd, name, t):
    return linear(sd, name, t.permute(0, 2, 3, 1)).permute(0, 3, 1, 2)


def tensornet_representation(sd, cfg, z, pos, batch, static_shapes=True, prefix="representation_model.",
                             hooks=None):
    p = lambda n: prefix + n
    H = cfg["embedding_dimension"]
    cl, cu = cfg["cutoff_lower"], cfg["cutoff_upper"]
    N = z.shape[0]
    src, dst, dl, r, _ = edge_geometry(pos, batch, cl, cu, max_pairs=cfg["max_num_neighbors"] * N,
                                       pad_static=static_shapes, box=cfg.get("box"))
    f = expnorm(r, sd[p("distance_expansion.means")], sd[p("distance_expansion.betas")], cl, cu)
    self_edge = src == dst
    u = dl / torch.where(self_edge, torch.ones_like(r), r).unsqueeze(1)
    C = cosine_cutoff(r, cl, cu)
    # TensorEmbedding (tensornet.py:287-326)
    te = p("tensor_embedding.")
    W1 = linear(sd, te + "distance_proj1", f) * C.unsqueeze(1)
    W2 = linear(sd, te + "distance_proj2", f) * C.unsqueeze(1)
    W3 = linear(sd, te + "distance_proj3", f) * C.unsqueeze(1)
    eye = torch.eye(3, dtype=pos.dtype)
    Iij = W1[..., None, None] * eye
    Aij = W2[..., None, None] * _skew(u)[:, None]
    Sij = W3[..., None, None] * _sym(u)[:, None]
    Z = sd[te + "emb.weight"][z]
    Zij = linear(sd, te + "emb2", torch.cat([Z.index_select(0, src), Z.index_select(0, dst)], dim=1))[..., None, None]
    I = torch.zeros(N, H, 3, 3, dtype=pos.dtype).index_add(0, src, Zij * Iij)
    A = torch.zeros(N, H, 3, 3, dtype=pos.dtype).index_add(0, src, Zij * Aij)
    S = torch.zeros(N, H, 3, 3, dtype=pos.dtype).index_add(0, src, Zij * Sij)
    norm = layer_norm(sd, te + "init_norm", _tnorm(I + A + S))
    I = _chan_linear(sd, te + "linears_tensor.0", I)
    A = _chan_linear(sd, te + "linears_tensor.1", A)
    S = _chan_linear(sd, te + "linears_tensor.2", S)
    for li in range(2):
        norm = F.silu(linear(sd, te + f"linears_scalar.{li}", norm))
    norm = norm.reshape(N, H, 3)
    X = I * norm[..., 0, None, None] + A * norm[..., 1, None, None] + S * norm[..., 2, None, None]
    group = cfg.get("equivariance_invariance_group", "O(3)")
    for li in range(cfg["num_layers"]):
        lp = p(f"layers.{li}.")
        ea = f
        for k in range(3):
            ea = F.silu(linear(sd, lp + f"linears_scalar.{k}", ea))
        ea = (ea * C.unsqueeze(1)).reshape(-1, H, 3)
        X = X / (_tnorm(X) + 1)[..., None, None]
        I, A, S = _decompose(X)
        I = _chan_linear(sd, lp + "linears_tensor.0", I)
        A = _chan_linear(sd, lp + "linears_tensor.1", A)
        S = _chan_linear(sd, lp + "linears_tensor.2", S)
        Y = I + A + S
        zero = torch.zeros(N, H, 3, 3, dtype=pos.dtype)
        Im = zero.index_add(0, src, ea[..., 0, None, None] * I.index_select(0, dst))
        Am = zero.index_add(0, src, ea[..., 1, None, None] * A.index_select(0, dst))
        Sm = zero.index_add(0, src, ea[..., 2, None, None] * S.index_select(0, dst))
        msg = Im + Am + Sm
        if group == "O(3)":
            I, A, S = _decompose(torch.matmul(msg, Y) + torch.matmul(Y, msg))
        else:
            I, A, S = _decompose(2 * torch.matmul(Y, msg))
        normp1 = (_tnorm(I + A + S) + 1)[..., None, None]
        I, A, S = I / normp1, A / normp1, S / normp1
        I = _chan_linear(sd, lp + "linears_tensor.3", I)
        A = _chan_linear(sd, lp + "linears_tensor.4", A)
        S = _chan_linear(sd, lp + "linears_tensor.5", S)
        dX = I + A + S
        X = X + dX + torch.matmul(dX, dX)
        if hooks is not None:
            hooks[f"layer{li}/X"] = X
    I, A, S = _decompose(X)
    x = torch.cat((_tnorm(I), _tnorm(A), _tnorm(S)), dim=-1)
    x = layer_norm(sd, p("out_norm"), x)
    return F.silu(linear(sd, p("linear"), x))


# ----------------------------------------------------------------------------- full model
def energy_forces(sd, cfg, z, pos, batch, dtype=torch.float64, static_shapes=True, create_graph=False,
                  hooks=None):
    """TorchMD_Net.forward with derivative=True (model.py:232-300) for ET (EquivariantScalar head)
    or TensorNet (Scalar head).  ``sd``: state_dict (tensors or numpy).  Returns (y, neg_dy)."""
    def conv(v):
        if torch.is_tensor(v):
            v = v.cpu()
            if v.requires_grad:  # keep the autograd link (parameter gradients, double backward)
                return v.to(dtype)
            v = v.detach()
        else:
            v = torch.as_tensor(np.asarray(v))
        return v.to(dtype) if v.is_floating_point() else v
    sd = {k: conv(v) for k, v in sd.items()}
    z = torch.as_tensor(z).long().cpu()
    batch = torch.as_tensor(batch).long().cpu()
    pos = torch.as_tensor(pos).detach().cpu().to(dtype).clone().requires_grad_(True)
    if cfg["model"] == "equivariant-transformer":
        x, v = et_representation(sd, cfg, z, pos, batch, hooks=hooks)
        x = equivariant_scalar(sd, cfg, x, v)
    else:
        x = tensornet_representation(sd, cfg, z, pos, batch, static_shapes=static_shapes, hooks=hooks)
        x = scalar_head(sd, x)
    x = x * sd.get("std", torch.ones((), dtype=dtype))
    if "prior_model.0.atomref.weight" in sd:
        x = x + sd["prior_model.0.atomref.weight"][z]
    nmol = int(batch.max()) + 1
    y = torch.zeros(nmol, 1, dtype=dtype).index_add(0, batch, x) + sd.get("mean", torch.zeros((), dtype=dtype))
    dy = torch.autograd.grad(y.sum(), pos, create_graph=create_graph)[0]
    return y, -dy


def qm9_like(n_mol, gen_seed=1):
    """SURVEY.md §8(d) QM9-like synthetic molecules (same generator as the fixture script)."""
    g = torch.Generator().manual_seed(gen_seed)
    zs, ps, bs = [], [], []
    for m in range(n_mol):
        n = int(torch.randint(9, 30, (1,), generator=g))
        heavy = n // 2
        zz = torch.ones(n, dtype=torch.long)
        zz[:heavy] = torch.tensor([6, 7, 8, 9])[torch.randint(0, 4, (heavy,), generator=g)]
        zs.append(zz)
        ps.append(torch.randn(n, 3, generator=g, dtype=torch.float64) * 1.6)
        bs.append(torch.full((n,), m, dtype=torch.long))
    return torch.cat(zs), torch.cat(ps), torch.cat(bs)
