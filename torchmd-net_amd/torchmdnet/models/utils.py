"""Model building blocks (mirror of the reference ``torchmdnet/models/utils.py`` API).

Class names, constructor arguments, parameter/buffer names and parameter-initialisation order
follow the reference so that checkpoints (state_dict keys) and ``torch.manual_seed`` reproduce the
same weights.  The compute of the hot-path blocks is delegated to the HIP kernels in
``torchmdnet.kernels``:
  * OptimizedDistance       -> torchmdnet_neighbors::get_neighbor_pairs (HIP, tmdnet_nl_build)
  * ExpNormal/GaussianSmearing, CosineCutoff -> tmdnet_edge_geom_fwd/bwd (on GPU tensors)
  * NeighborEmbedding       -> tmdnet_nbr_embed_fwd/bwd
"""
import math
import warnings
from typing import Optional, Tuple

import torch
import torch.nn.functional as F
from torch import Tensor, nn

from .. import _native as nat
from .. import kernels
from ..neighbors import get_neighbor_pairs_kernel


class CosineCutoff(nn.Module):
    """Reference utils.py:362-390."""

    def __init__(self, cutoff_lower=0.0, cutoff_upper=5.0):
        super().__init__()
        self.cutoff_lower = cutoff_lower
        self.cutoff_upper = cutoff_upper

    def forward(self, distances: Tensor) -> Tensor:
        if torch.jit.is_scripting():
            return _cos_cut(distances, float(self.cutoff_lower), float(self.cutoff_upper))
        nat.require_gpu(distances, "CosineCutoff")
        return _rbf_cutoff_only(distances, self.cutoff_lower, self.cutoff_upper)


def _graph_from_dist(dist):
    """Minimal graph for edge-geometry kernels evaluated on a bare distance vector."""
    z = torch.zeros(dist.shape[0], dtype=torch.int32, device=dist.device)
    o = torch.ones(dist.shape[0], dtype=torch.int32, device=dist.device)
    g = kernels.EdgeGraph(0, None, z, o, None, None, None, dist.shape[0], False)
    return g


def _rbf_cutoff_only(dist, cl, cu):
    flat = dist.reshape(-1).contiguous()
    g = _graph_from_dist(flat)
    dl = torch.zeros((flat.shape[0], 3), dtype=flat.dtype, device=flat.device)
    dummy = torch.zeros(1, dtype=flat.dtype, device=flat.device)
    _, C, _ = kernels._EdgeGeom.apply(dl, flat, g, dummy, dummy, float(cl), float(cu),
                                      nat.RBF_EXPNORM, (False, True, False))
    return C.view(dist.shape)


class GaussianSmearing(nn.Module):
    """Reference utils.py:272-300."""

    def __init__(self, cutoff_lower=0.0, cutoff_upper=5.0, num_rbf=50, trainable=True, dtype=torch.float32):
        super().__init__()
        self.cutoff_lower = cutoff_lower
        self.cutoff_upper = cutoff_upper
        self.num_rbf = num_rbf
        self.trainable = trainable
        self.dtype = dtype
        offset, coeff = self._initial_params()
        if trainable:
            self.register_parameter("coeff", nn.Parameter(coeff))
            self.register_parameter("offset", nn.Parameter(offset))
        else:
            self.register_buffer("coeff", coeff)
            self.register_buffer("offset", offset)

    rbf_type = nat.RBF_GAUSS
    __constants__ = ["rbf_type"]

    def _initial_params(self):
        offset = torch.linspace(self.cutoff_lower, self.cutoff_upper, self.num_rbf, dtype=self.dtype)
        coeff = -0.5 / (offset[1] - offset[0]) ** 2
        return offset, coeff

    def reset_parameters(self):
        offset, coeff = self._initial_params()
        self.offset.data.copy_(offset)
        self.coeff.data.copy_(coeff)

    def kernel_params(self):
        return self.offset, self.coeff.reshape(1).expand(self.num_rbf).contiguous()

    def forward(self, dist: Tensor) -> Tensor:
        if torch.jit.is_scripting():  # reference utils.py:298-300
            d = dist.unsqueeze(-1) - self.offset
            return torch.exp(self.coeff * torch.pow(d, 2))
        nat.require_gpu(dist, "GaussianSmearing")
        if self.trainable and torch.is_grad_enabled():
            d = dist.unsqueeze(-1) - self.offset
            return torch.exp(self.coeff * torch.pow(d, 2))
        return _rbf_only(self, dist)


class ExpNormalSmearing(nn.Module):
    """Reference utils.py:303-344 (PhysNet expnorm basis)."""

    rbf_type = nat.RBF_EXPNORM
    __constants__ = ["rbf_type"]

    def __init__(self, cutoff_lower=0.0, cutoff_upper=5.0, num_rbf=50, trainable=True, dtype=torch.float32):
        super().__init__()
        self.cutoff_lower = cutoff_lower
        self.cutoff_upper = cutoff_upper
        self.num_rbf = num_rbf
        self.trainable = trainable
        self.dtype = dtype
        self.cutoff_fn = CosineCutoff(0, cutoff_upper)
        self.alpha = 5.0 / (cutoff_upper - cutoff_lower)
        means, betas = self._initial_params()
        if trainable:
            self.register_parameter("means", nn.Parameter(means))
            self.register_parameter("betas", nn.Parameter(betas))
        else:
            self.register_buffer("means", means)
            self.register_buffer("betas", betas)

    def _initial_params(self):
        start_value = torch.exp(torch.scalar_tensor(-self.cutoff_upper + self.cutoff_lower, dtype=self.dtype))
        means = torch.linspace(start_value, 1, self.num_rbf, dtype=self.dtype)
        betas = torch.tensor([(2 / self.num_rbf * (1 - start_value)) ** -2] * self.num_rbf, dtype=self.dtype)
        return means, betas

    def reset_parameters(self):
        means, betas = self._initial_params()
        self.means.data.copy_(means)
        self.betas.data.copy_(betas)

    def kernel_params(self):
        return self.means, self.betas

    def forward(self, dist: Tensor) -> Tensor:
        if torch.jit.is_scripting():  # reference utils.py:339-344
            d = dist.unsqueeze(-1)
            return _cos_cut(d, 0.0, float(self.cutoff_upper)) * torch.exp(
                -self.betas * (torch.exp(self.alpha * (-d + self.cutoff_lower)) - self.means) ** 2)
        nat.require_gpu(dist, "ExpNormalSmearing")
        if self.trainable and torch.is_grad_enabled():
            d = dist.unsqueeze(-1)
            return _cos_cut(d, 0.0, self.cutoff_upper) * torch.exp(
                -self.betas * (torch.exp(self.alpha * (-d + self.cutoff_lower)) - self.means) ** 2)
        return _rbf_only(self, dist)


def _cos_cut(r: Tensor, cl: float, cu: float) -> Tensor:
    """CosineCutoff in ATen ops (reference utils.py:368-390)."""
    if cl > 0:
        c = 0.5 * (torch.cos(math.pi * (2 * (r - cl) / (cu - cl) + 1.0)) + 1.0)
        return c * (r < cu).to(r.dtype) * (r > cl).to(r.dtype)
    return 0.5 * (torch.cos(r * math.pi / cu) + 1.0) * (r < cu).to(r.dtype)


def _rbf_only(module, dist):
    flat = dist.reshape(-1).contiguous()
    g = _graph_from_dist(flat)
    dl = torch.zeros((flat.shape[0], 3), dtype=flat.dtype, device=flat.device)
    mu, beta = module.kernel_params()
    f, _, _ = kernels._EdgeGeom.apply(dl, flat, g, mu.detach().to(flat.dtype).contiguous(),
                                      beta.detach().to(flat.dtype).contiguous(),
                                      float(module.cutoff_lower), float(module.cutoff_upper),
                                      module.rbf_type, (True, False, False))
    return f.view(*dist.shape, module.num_rbf)


class ShiftedSoftplus(nn.Module):
    def __init__(self):
        super().__init__()
        self.shift = torch.log(torch.tensor(2.0)).item()

    def forward(self, x):
        return F.softplus(x) - self.shift


class OptimizedDistance(torch.nn.Module):
    """Neighbour list module (reference utils.py:112-269), backed by the HIP neighbour op.

    Same constructor, same forward contract: returns (edge_index, edge_weight, edge_vec|None),
    trimmed to the found pairs when ``resize_to_fit`` (host sync, as the reference), otherwise padded
    with (-1, -1) / 0 to ``max_num_pairs``.  ``graph(pos, batch)`` additionally returns the CSR
    EdgeGraph used by the fused model kernels.
    """

    def __init__(self, cutoff_lower=0.0, cutoff_upper=5.0, max_num_pairs=-32, return_vecs=False,
                 loop=False, strategy="brute", include_transpose=True, resize_to_fit=True,
                 check_errors=True, box=None, long_edge_index=True):
        super().__init__()
        self.cutoff_upper = cutoff_upper
        self.cutoff_lower = cutoff_lower
        self.max_num_pairs = max_num_pairs
        self.strategy = strategy
        self.box: Optional[Tensor] = box
        self.loop = loop
        self.return_vecs = return_vecs
        self.include_transpose = include_transpose
        self.resize_to_fit = resize_to_fit
        self.use_periodic = True
        if self.box is None:
            self.use_periodic = False
            self.box = torch.empty((0, 0))
            if self.strategy == "cell":
                lbox = cutoff_upper * 3.0
                self.box = torch.tensor([[lbox, 0, 0], [0, lbox, 0], [0, 0, lbox]])
        self.box = self.box.cpu()
        self.check_errors = check_errors
        self.long_edge_index = long_edge_index
        # HIP-graph mode (torchmdnet.graphs): fixed edge capacity, no host synchronisation
        self.static_capacity = None
        # graph(): number the edge pairs in the build itself (the ET consumer sets it; sorted rows)
        self.pair_rows = False

    def _max_pairs(self, n: int) -> int:
        return -self.max_num_pairs * n if self.max_num_pairs < 0 else self.max_num_pairs

    def forward(self, pos: Tensor, batch: Optional[Tensor] = None) -> Tuple[Tensor, Tensor, Optional[Tensor]]:
        self.box = self.box.to(pos.dtype)
        max_pairs = self._max_pairs(pos.shape[0])
        if batch is None:
            batch = torch.zeros(pos.shape[0], dtype=torch.long, device=pos.device)
        edge_index, edge_vec, edge_weight, num_pairs = get_neighbor_pairs_kernel(
            strategy=self.strategy, positions=pos, batch=batch, max_num_pairs=max_pairs,
            cutoff_lower=self.cutoff_lower, cutoff_upper=self.cutoff_upper, loop=self.loop,
            include_transpose=self.include_transpose, box_vectors=self.box,
            use_periodic=self.use_periodic)
        if self.check_errors:
            if num_pairs[0] > max_pairs:
                raise RuntimeError("Found num_pairs({}) > max_num_pairs({})".format(num_pairs[0], max_pairs))
        if self.resize_to_fit:
            mask = edge_index[0] != -1
            edge_index = edge_index[:, mask]
            edge_weight = edge_weight[mask]
            edge_vec = edge_vec[mask, :]
        if self.long_edge_index:
            edge_index = edge_index.to(torch.long)
        if self.return_vecs:
            return edge_index, edge_weight, edge_vec
        return edge_index, edge_weight, None

    def graph(self, pos: Tensor, batch: Optional[Tensor] = None):
        """Symmetric CSR EdgeGraph (loop as configured) for the fused model kernels."""
        if not self.include_transpose:
            raise RuntimeError("the fused model path needs include_transpose=True")
        if batch is None:
            batch = torch.zeros(pos.shape[0], dtype=torch.long, device=pos.device)
        box = self.box.to(pos.dtype) if self.use_periodic else None
        strategy = self.strategy
        if strategy == "cell" and not self.use_periodic:
            box = None
        g = kernels.build_graph(pos, batch, self.cutoff_lower, self.cutoff_upper,
                                self._max_pairs(pos.shape[0]), loop=self.loop, strategy=strategy,
                                box=box, check_errors=self.check_errors,
                                static_capacity=self.static_capacity, pairs=self.pair_rows)
        # keep only the device-side status of the last build (static-capacity overflow flag, pair
        # count): holding the graph itself would keep its autograd history -- and the positions'
        # AccumulateGrad node -- alive across steps, which breaks HIP-graph capture of later steps
        self.last_overflow = getattr(g, "overflow", None)
        self.last_num_pairs = g.num_pairs_dev if g.num_pairs_dev is not None else g.num_pairs
        return g


class NeighborEmbedding(nn.Module):
    """Reference utils.py:43-108 (ET neighbour embedding, eq. 3 of arXiv:2202.02541).

    forward(z, x, edge_index, edge_weight, edge_attr): ``edge_index`` may be a (2, E) tensor (any
    symmetric edge list) or the model's CSR EdgeGraph (fast path).
    """

    def __init__(self, hidden_channels, num_rbf, cutoff_lower, cutoff_upper, max_z=100, dtype=torch.float32):
        super().__init__()
        self.embedding = nn.Embedding(max_z, hidden_channels, dtype=dtype)
        self.distance_proj = nn.Linear(num_rbf, hidden_channels, dtype=dtype)
        self.combine = nn.Linear(hidden_channels * 2, hidden_channels, dtype=dtype)
        self.cutoff = CosineCutoff(cutoff_lower, cutoff_upper)
        self.reset_parameters()

    def jittable(self):
        return self

    def reset_parameters(self):
        self.embedding.reset_parameters()
        nn.init.xavier_uniform_(self.distance_proj.weight)
        nn.init.xavier_uniform_(self.combine.weight)
        self.distance_proj.bias.data.fill_(0)
        self.combine.bias.data.fill_(0)

    def script_forward(self, z: Tensor, x: Tensor, row_ptr: Tensor, src: Tensor, dst: Tensor, edge_attr: Tensor,
                       C: Tensor) -> Tensor:
        """TorchScript path: reference utils.py:90-108 with the aggregation as ``tmdnet::nbr_embed``."""
        W = self.distance_proj(edge_attr)
        x_nb = torch.ops.tmdnet.nbr_embed(self.embedding(z), W, C, row_ptr, src, dst)
        return self.combine(torch.cat([x, x_nb], dim=1))

    @torch.jit.unused
    def fused_forward(self, z: Tensor, x: Tensor, graph, r: Tensor, cutoff: Tensor, x_emb: Optional[Tensor],
                      rbf, rbf_fn) -> Tensor:
        """Large systems (TorchMD_ET): distance_proj formed inside the aggregation kernel from the distances
        ``r`` (kernels.nbr_embed_fused; ``rbf`` = (mu, beta, cutoff_lower, cutoff_upper, rbf_type), ``rbf_fn``
        the basis module) -- no rbf or projection rows; the model's CSR graph and cutoff."""
        if x_emb is None:
            x_emb = self.embedding(z)
        x_cat = kernels.nbr_embed_fused(x_emb, r, cutoff, self.distance_proj.weight, self.distance_proj.bias,
                                        graph, rbf, rbf_fn, x_self=x)
        return kernels.linear(x_cat, self.combine.weight, self.combine.bias)

    def forward(self, z: Tensor, x: Tensor, edge_index: Tensor, edge_weight: Tensor, edge_attr: Tensor,
                cutoff: Optional[Tensor] = None, x_emb: Optional[Tensor] = None) -> Tensor:
        """``x_emb``: this module's embedding of ``z`` when the caller looked it up already (TorchMD_ET
        does both tables' lookups in one node)."""
        if torch.jit.is_scripting():
            raise RuntimeError("scripted NeighborEmbedding: use script_forward (CSR graph)")
        graph, perm = as_graph(edge_index, x.shape[0])
        if perm is not None:
            edge_weight, edge_attr = edge_weight[perm], edge_attr[perm]
        C = cutoff if cutoff is not None else self.cutoff(edge_weight)
        if x_emb is None:
            x_emb = self.embedding(z)
        if x.is_cuda:  # Linears with hand-written (TN GEMM) weight gradients, also in the second order
            W = kernels.linear(edge_attr, self.distance_proj.weight, self.distance_proj.bias)
            return kernels.linear(kernels.nbr_embed(x_emb, W, C, graph, x_self=x), self.combine.weight,
                                  self.combine.bias)
        W = self.distance_proj(edge_attr)
        # [x | x_nb] comes out of the aggregation kernel itself (no concatenation launch)
        return self.combine(kernels.nbr_embed(x_emb, W, C, graph, x_self=x))


def as_graph(edge_index, n_nodes):
    """EdgeGraph fast path, or a CSR view (+ permutation) of a reference-style edge_index."""
    if isinstance(edge_index, kernels.EdgeGraph):
        return edge_index, None
    g, perm = kernels.EdgeGraph.from_edge_index(edge_index, n_nodes)
    return g, perm


class GatedEquivariantBlock(nn.Module):
    """Reference utils.py:456-522 (Schuett et al. 2021 gated equivariant block)."""

    def __init__(self, hidden_channels, out_channels, intermediate_channels=None, activation="silu",
                 scalar_activation=False, dtype=torch.float):
        super().__init__()
        self.out_channels = out_channels
        if intermediate_channels is None:
            intermediate_channels = hidden_channels
        self.vec1_proj = nn.Linear(hidden_channels, hidden_channels, bias=False, dtype=dtype)
        self.vec2_proj = nn.Linear(hidden_channels, out_channels, bias=False, dtype=dtype)
        act_class = act_class_mapping[activation]
        self.update_net = nn.Sequential(
            nn.Linear(hidden_channels * 2, intermediate_channels, dtype=dtype),
            act_class(),
            nn.Linear(intermediate_channels, out_channels * 2, dtype=dtype),
        )
        self.act = act_class() if scalar_activation else None

    def reset_parameters(self):
        nn.init.xavier_uniform_(self.vec1_proj.weight)
        nn.init.xavier_uniform_(self.vec2_proj.weight)
        nn.init.xavier_uniform_(self.update_net[0].weight)
        self.update_net[0].bias.data.fill_(0)
        nn.init.xavier_uniform_(self.update_net[2].weight)
        self.update_net[2].bias.data.fill_(0)

    def forward(self, x, v):
        # zero rows (isolated atoms) are excluded from the norm so their gradient is not NaN; the
        # reference does this with a host-synchronising boolean mask (utils.py:499-512), this is the
        # sync-free equivalent (same values, same zero gradients on those rows)
        vec1 = kernels.masked_norm(self.vec1_proj(v))
        vec2 = self.vec2_proj(v)
        x = torch.cat([x, vec1], dim=-1)
        x, v = torch.split(self.update_net(x), self.out_channels, dim=-1)
        v = v.unsqueeze(1) * vec2
        if self.act is not None:
            x = self.act(x)
        return x, v


rbf_class_mapping = {"gauss": GaussianSmearing, "expnorm": ExpNormalSmearing}

act_class_mapping = {
    "ssp": ShiftedSoftplus,
    "silu": nn.SiLU,
    "tanh": nn.Tanh,
    "sigmoid": nn.Sigmoid,
}

dtype_mapping = {16: torch.float16, 32: torch.float, 64: torch.float64}


class Distance(nn.Module):
    """torch_cluster radius_graph wrapper of the reference (utils.py:393-453) -- used only by the
    Graph-Network / Transformer models, which are outside this package's scope."""

    def __init__(self, *args, **kwargs):
        raise NotImplementedError("Distance (torch_cluster) is not part of the ET/TensorNet hot path; "
                                  "use OptimizedDistance")


def check_stream_capturing():
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()
