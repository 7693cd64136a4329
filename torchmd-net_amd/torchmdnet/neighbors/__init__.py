"""``torchmdnet_neighbors::get_neighbor_pairs`` -- the reference's native op, same schema.

Reference: torchmdnet/neighbors/neighbors.cpp:3-5 (schema), neighbors/__init__.py:1-17 (loader),
neighbors_cuda.cu:25-89 (CUDA + AutogradCUDA registration).  Here the op is registered with
``torch.library`` on the CUDA (= HIP on ROCm) and AutogradCUDA keys and its compute is the HIP
library (``tmdnet_nl_build``).  Returned values, as in the reference: (neighbors int32 [2, P],
deltas [P, 3], distances [P], num_pairs int32 [1]) with P = max_num_pairs, padded with (-1, -1)/0.

There is deliberately no CPU kernel: calling the op with CPU tensors raises.
"""
import torch

from .. import kernels

_SCHEMA = ("get_neighbor_pairs(str strategy, Tensor positions, Tensor batch, Tensor box_vectors, "
           "bool use_periodic, Scalar cutoff_lower, Scalar cutoff_upper, Scalar max_num_pairs, "
           "bool loop, bool include_transpose) -> (Tensor neighbors, Tensor distances, "
           "Tensor distance_vecs, Tensor num_pairs)")


def _forward(strategy, positions, batch, box_vectors, use_periodic, cutoff_lower, cutoff_upper,
             max_num_pairs, loop, include_transpose):
    if use_periodic:
        kernels.validate_box(box_vectors, cutoff_upper)
    if strategy == "brute" and positions.shape[0] >= 32768:
        strategy = "shared"  # reference neighbors_cuda.cu:81-83 (same kernel family here)
    nb, dl, dist, num, _, _ = kernels.neighbor_pairs_raw(
        strategy, positions, batch, box_vectors, use_periodic, float(cutoff_lower), float(cutoff_upper),
        int(max_num_pairs), loop, include_transpose, pad_output=True, want_csr=False)
    return nb, dl, dist, num


class _NeighborPairs(torch.autograd.Function):
    """Reference NeighborAutograd (neighbors_cuda.cu:25-72): backward written with differentiable
    index_add_ so it can be differentiated twice."""

    @staticmethod
    def forward(ctx, strategy, positions, batch, box_vectors, use_periodic, cutoff_lower,
                cutoff_upper, max_num_pairs, loop, include_transpose):
        nb, dl, dist, num = _forward(strategy, positions, batch, box_vectors, use_periodic,
                                     cutoff_lower, cutoff_upper, max_num_pairs, loop, include_transpose)
        ctx.save_for_backward(nb, dl, dist)
        ctx.num_atoms = positions.shape[0]
        ctx.mark_non_differentiable(nb, num)
        return nb, dl, dist, num

    @staticmethod
    def backward(ctx, _gnb, grad_edge_vec, grad_edge_weight, _gnum):
        edge_index, edge_vec, edge_weight = ctx.saved_tensors
        n = ctx.num_atoms
        if grad_edge_vec is None:
            grad_edge_vec = torch.zeros_like(edge_vec)
        if grad_edge_weight is None:
            grad_edge_weight = torch.zeros_like(edge_weight)
        zero_mask = edge_weight == 0
        zero_mask3 = zero_mask.unsqueeze(-1).expand_as(grad_edge_vec)
        grad_distances_ = (edge_vec / edge_weight.masked_fill(zero_mask, 1).unsqueeze(-1)
                           * grad_edge_weight.masked_fill(zero_mask, 0).unsqueeze(-1))
        result = grad_edge_vec.masked_fill(zero_mask3, 0) + grad_distances_
        grad_positions_ = torch.zeros((n + 1, 3), dtype=edge_vec.dtype, device=edge_vec.device)
        edge_index_ = edge_index.long().masked_fill(zero_mask.unsqueeze(0).expand_as(edge_index), n)
        edge_index_ = edge_index_.masked_fill(edge_index_ < 0, n)
        grad_positions_ = grad_positions_.index_add(0, edge_index_[0], result)
        grad_positions_ = grad_positions_.index_add(0, edge_index_[1], -result)
        return None, grad_positions_[:n], None, None, None, None, None, None, None, None


_lib = torch.library.Library("torchmdnet_neighbors", "DEF")
_lib.define(_SCHEMA)


def _cuda_impl(strategy, positions, batch, box_vectors, use_periodic, cutoff_lower, cutoff_upper,
               max_num_pairs, loop, include_transpose):
    return _forward(strategy, positions, batch, box_vectors, use_periodic, cutoff_lower,
                    cutoff_upper, max_num_pairs, loop, include_transpose)


def _autograd_impl(strategy, positions, batch, box_vectors, use_periodic, cutoff_lower, cutoff_upper,
                   max_num_pairs, loop, include_transpose):
    return _NeighborPairs.apply(strategy, positions, batch, box_vectors, use_periodic, cutoff_lower,
                                cutoff_upper, max_num_pairs, loop, include_transpose)


def _cpu_impl(*args, **kwargs):
    raise RuntimeError("torchmd-net_amd: get_neighbor_pairs runs only on a ROCm GPU (CPU tensors given)")


_lib.impl("get_neighbor_pairs", _cuda_impl, "CUDA")
_lib.impl("get_neighbor_pairs", _autograd_impl, "AutogradCUDA")
_lib.impl("get_neighbor_pairs", _cpu_impl, "CPU")

get_neighbor_pairs_kernel = torch.ops.torchmdnet_neighbors.get_neighbor_pairs

try:  # reference neighbors/__init__.py:15-17
    import torch._dynamo as dynamo
    dynamo.disallow_in_graph(get_neighbor_pairs_kernel)
except Exception:  # pragma: no cover
    pass
