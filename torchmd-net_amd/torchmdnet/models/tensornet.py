"""TensorNet (mirror of reference ``torchmdnet/models/tensornet.py``; Simeon & De Fabritiis 2023).

Module tree, parameter names and initialisation order follow the reference (tensornet.py:70-410).
Edge work runs in HIP kernels (``tmdnet_tn_embed_*``, ``tmdnet_tn_message_*``): the per-edge
``emb2(cat(Z_i, Z_j))`` of TensorEmbedding is split into two per-node GEMM halves and the
scatter over ``edge_index[0]`` becomes a CSR walk of the reversed rows (no atomics).
``static_shapes=True`` (the reference default) reproduces the reference CUDA semantics: padded
neighbour slots become extra (0, 0) edges with r = 0 (tensornet.py:215-221), applied here as a
multiplicity on atom 0's self loop.
"""
import os
from typing import List, Optional, Tuple

import torch
from torch import Tensor, nn

from .. import kernels, tn_node
from .utils import CosineCutoff, OptimizedDistance, act_class_mapping, as_graph, rbf_class_mapping

# reference tensornet.py:13-14 sets TF32 matmul globally; gfx950 has no TF32/xf32 path, so fp32
# GEMMs stay exact fp32 here.

# Large systems (C5: the 50k-atom water box, ~2M edges): the Interaction's edge MLP (reference
# tensornet.py:381-385, a function of |r| only) runs once per edge PAIR -- (E + N) / 2 rows instead of E --
# on the x3 GEMM with SiLU / cutoff epilogues, and the message reads the pair rows (tmdnet_tn_message_*_pairs).
# From this many edges on; TMDNET_TN_PAIRS=0 keeps per-edge rows (A/B).
PAIR_MIN_EDGES = 131072
PAIRS = os.environ.get("TMDNET_TN_PAIRS", "1") != "0"


def vector_to_skewtensor(vector):
    return kernels._skew(vector).squeeze(0)


def vector_to_symtensor(vector):
    return kernels._sym(vector)


def decompose_tensor(tensor):
    I = (tensor.diagonal(offset=0, dim1=-1, dim2=-2)).mean(-1)[..., None, None] * torch.eye(
        3, 3, device=tensor.device, dtype=tensor.dtype)
    A = 0.5 * (tensor - tensor.transpose(-2, -1))
    S = 0.5 * (tensor + tensor.transpose(-2, -1)) - I
    return I, A, S


def new_radial_tensor(I, A, S, f_I, f_A, f_S):
    return f_I[..., None, None] * I, f_A[..., None, None] * A, f_S[..., None, None] * S


def tensor_norm(tensor):
    return (tensor ** 2).sum((-2, -1))


# ----------------------------------------------------------------------------- TorchScript path
# Compact-tensor algebra in ATen ops (tn_node.op_composite, written for TorchScript): the scripted
# model runs the edge work through the tmdnet::tn_embed / tmdnet::tn_message operators (HIP, C++
# autograd) and this node algebra through ATen.
def _s_full9(c: Tensor) -> Tensor:
    i, a01, a02, a12, s00, s11, s01, s02, s12 = c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7], c[8]
    F = torch.stack((i + s00, a01 + s01, a02 + s02, s01 - a01, i + s11, a12 + s12,
                     s02 - a02, s12 - a12, i - s00 - s11), dim=-1)
    return F.view(F.shape[0], F.shape[1], 3, 3)


def _s_decomp9(X: Tensor) -> Tensor:
    f = X.reshape(X.shape[0], X.shape[1], 9)
    i = (f[..., 0] + f[..., 4] + f[..., 8]) / 3
    return torch.stack((i, 0.5 * (f[..., 1] - f[..., 3]), 0.5 * (f[..., 2] - f[..., 6]),
                        0.5 * (f[..., 5] - f[..., 7]), f[..., 0] - i, f[..., 4] - i,
                        0.5 * (f[..., 1] + f[..., 3]), 0.5 * (f[..., 2] + f[..., 6]),
                        0.5 * (f[..., 5] + f[..., 7])), dim=0)


def _s_mm33(a: Tensor, b: Tensor) -> Tensor:
    return (a.unsqueeze(-1) * b.unsqueeze(-3)).sum(-2)


def _s_tnorm(t: Tensor) -> Tensor:
    return (t ** 2).sum((-2, -1))


def _s_mix3(c: Tensor, w0: Tensor, w1: Tensor, w2: Tensor) -> Tensor:
    return torch.cat((torch.matmul(c[0:1], w0.t()), torch.matmul(c[1:4], w1.t()),
                      torch.matmul(c[4:9], w2.t())), dim=0)


class TensorNet(nn.Module):
    __jit_ignored_attributes__ = ["_pad_shift"]  # host-side padded-training state (eager path only)

    def __init__(self, hidden_channels=128, num_layers=2, num_rbf=32, rbf_type="expnorm",
                 trainable_rbf=False, activation="silu", cutoff_lower=0, cutoff_upper=4.5,
                 max_num_neighbors=64, max_z=128, equivariance_invariance_group="O(3)",
                 static_shapes=True, dtype=torch.float32):
        super().__init__()
        assert rbf_type in rbf_class_mapping, (
            f'Unknown RBF type "{rbf_type}". Choose from {", ".join(rbf_class_mapping.keys())}.')
        assert activation in act_class_mapping, (
            f'Unknown activation function "{activation}". Choose from {", ".join(act_class_mapping.keys())}.')
        assert equivariance_invariance_group in ["O(3)", "SO(3)"], (
            f'Unknown group "{equivariance_invariance_group}". Choose O(3) or SO(3).')
        self.hidden_channels = hidden_channels
        self.equivariance_invariance_group = equivariance_invariance_group
        self.num_layers = num_layers
        self.num_rbf = num_rbf
        self.rbf_type = rbf_type
        self.activation = activation
        self.cutoff_lower = cutoff_lower
        self.cutoff_upper = cutoff_upper
        self.trainable_rbf = trainable_rbf
        act_class = act_class_mapping[activation]
        self.distance_expansion = rbf_class_mapping[rbf_type](cutoff_lower, cutoff_upper, num_rbf, trainable_rbf)
        self.tensor_embedding = TensorEmbedding(hidden_channels, num_rbf, act_class, cutoff_lower,
                                                cutoff_upper, trainable_rbf, max_z, dtype)
        self.layers = nn.ModuleList()
        if num_layers != 0:
            for _ in range(num_layers):
                self.layers.append(Interaction(num_rbf, hidden_channels, act_class, cutoff_lower, cutoff_upper,
                                               equivariance_invariance_group, dtype))
        self.linear = nn.Linear(3 * hidden_channels, hidden_channels, dtype=dtype)
        self.out_norm = nn.LayerNorm(3 * hidden_channels, dtype=dtype)
        self.act = act_class()
        self.static_shapes = static_shapes
        self.reorder_atoms = True
        # padded batches (training.PaddedBatches): (device int32 [1], host int) correction of the pair count
        # that keeps atom 0's static_shapes padding multiplicity that of the REAL atoms (ghosts excluded)
        self._pad_shift: Optional[Tuple[Tensor, int]] = None
        self.distance = OptimizedDistance(cutoff_lower, cutoff_upper, max_num_pairs=-max_num_neighbors,
                                          return_vecs=True, loop=True, check_errors=False,
                                          resize_to_fit=not self.static_shapes, long_edge_index=True)
        self.reset_parameters()

    def reset_parameters(self):
        self.tensor_embedding.reset_parameters()
        for layer in self.layers:
            layer.reset_parameters()
        self.linear.reset_parameters()
        self.out_norm.reset_parameters()

    def forward(self, z: Tensor, pos: Tensor, batch: Tensor, q: Optional[Tensor] = None,
                s: Optional[Tensor] = None) -> Tuple[Tensor, Optional[Tensor], Tensor, Tensor, Tensor]:
        if torch.jit.is_scripting():
            return self._forward_script(z, pos, batch), None, z, pos, batch
        if self.reorder_atoms and z.shape[0] >= kernels.REORDER_MIN_ATOMS:
            perm = kernels.spatial_permutation(pos, batch, self.cutoff_upper,
                                               self.distance.box if self.distance.use_periodic else None)
            inv = torch.empty_like(perm)
            ar = torch.arange(perm.numel(), device=perm.device)
            inv[perm] = ar
            if self.static_shapes:
                # the padding semantics single out the caller's atom 0 (padded slots become (0, 0) edges,
                # tensornet.py:215-221): keep it at index 0 by swapping it with the Morton-first atom (same
                # molecule: the batch stays sorted).  Device ops only (no sync; capturable).
                j = inv[0:1]
                perm = perm.clone()
                perm.index_put_((j,), perm[0:1].clone())
                perm[0] = 0
                inv[perm] = ar
            x = self._forward(z[perm], pos.index_select(0, perm), batch[perm])
            return x[inv], None, z, pos, batch
        return self._forward(z, pos, batch), None, z, pos, batch

    def fused_energy_forces(self, z: Tensor, pos: Tensor, batch: Tensor, head: List[Tensor], std: Tensor,
                            mean: Tensor) -> Tuple[Tensor, Tensor]:
        """(TorchMD_Net.fused_eval is ET-only; the same signature keeps the scripted TorchMD_Net uniform)"""
        raise RuntimeError("fused_energy_forces: TorchMD_ET only")

    def _forward_script(self, z: Tensor, pos: Tensor, batch: Tensor) -> Tensor:
        """TorchScript path: reference tensornet.py:200-232 over the libtmdnet_torch.so operators."""
        d = self.distance
        cap = d._max_pairs(pos.shape[0])
        row_ptr, src, dst, tr, deltas, dist, num_pairs = torch.ops.tmdnet.neighbor_graph(
            pos, batch, d.box, d.use_periodic, float(d.cutoff_lower), float(d.cutoff_upper), cap, d.loop,
            d.strategy, d.check_errors, -1)
        # static_shapes: the reference's padded slots are (0, 0) edges at r = 0 -- multiplicity of atom 0's
        # self loop (one host read of the pair count, as the reference's resize_to_fit=False path shapes)
        m = float(1 + max(0, cap - int(num_pairs.item()))) if self.static_shapes else 1.0
        de = self.distance_expansion
        mu, beta = de.kernel_params()
        trainable = self.trainable_rbf and torch.is_grad_enabled()
        f, C, u = torch.ops.tmdnet.edge_geometry(deltas, dist, src, dst, mu, beta, float(self.cutoff_lower),
                                                 float(self.cutoff_upper), de.rbf_type, not trainable)
        if trainable:
            f = de(dist)
        X = self.tensor_embedding.script_forward(z, row_ptr, src, dst, f, C, u, m)
        for layer in self.layers:
            X = layer.script_forward(X, row_ptr, src, dst, f, C, m)
        c = _s_decomp9(X)
        nI = 3 * c[0] ** 2
        nA = 2 * (c[1] ** 2 + c[2] ** 2 + c[3] ** 2)
        nS = c[4] ** 2 + c[5] ** 2 + (c[4] + c[5]) ** 2 + 2 * (c[6] ** 2 + c[7] ** 2 + c[8] ** 2)
        x = self.out_norm(torch.cat((nI, nA, nS), dim=-1))
        return self.act(self.linear(x))

    def _forward(self, z: Tensor, pos: Tensor, batch: Tensor) -> Tensor:
        graph = self.distance.graph(pos, batch)
        cap = self.distance._max_pairs(pos.shape[0])
        shift = self._pad_shift
        if self.static_shapes and graph.static:
            # capture mode: the padding count stays on the device (no host sync)
            npd = graph.num_pairs_dev if shift is None else graph.num_pairs_dev + shift[0]
            graph.self0_dev = (npd, cap)
        elif self.static_shapes:
            n_eff = graph.num_pairs + (0 if shift is None else shift[1])
            graph.self0_mult = float(1 + max(0, cap - n_eff))
        else:  # (no padding multiplicity: the host pair count is not needed, e.g. under capture)
            graph.self0_mult = 1.0
        de = self.distance_expansion
        k = 1 + len(self.layers)  # consumers of the rbf / cutoff rows: the embedding and every layer
        if self.trainable_rbf and torch.is_grad_enabled():
            edge_attr = de(graph.distances)
            _, C, edge_vec = kernels.edge_geometry(graph, *de.kernel_params(), self.cutoff_lower,
                                                   self.cutoff_upper, de.rbf_type, want=(False, True, True))
            fs, Cs = [edge_attr], [C]
        else:
            # one alias per consumer (up to 3): their gradients are summed in the geometry backward kernel
            fs, Cs, edge_vec = kernels.edge_geometry(graph, *de.kernel_params(), self.cutoff_lower, self.cutoff_upper,
                                                     de.rbf_type, fan=(min(k, 3), min(k, 3)))
        pick = lambda t, i: t[min(i, len(t) - 1)]  # noqa: E731
        graph.cutoff = pick(Cs, 0)
        X = self.tensor_embedding(z, graph, graph.distances, edge_vec, pick(fs, 0))
        for i, layer in enumerate(self.layers):
            graph.cutoff = pick(Cs, i + 1)
            X = layer(X, graph, graph.distances, pick(fs, i + 1))
        x = tn_node.norms(X)  # cat(|I|^2, |A|^2, |S|^2) of decompose_tensor(X), one fused pass
        x = kernels.layer_norm(x, self.out_norm.weight, self.out_norm.bias, self.out_norm.eps)
        return kernels.mlp_act(x, [self.linear.weight], [self.linear.bias], self.act)


def _check_symmetric_graph(edge_index, n):
    graph, perm = as_graph(edge_index, n)
    return graph, perm


class TensorEmbedding(nn.Module):
    __jit_ignored_attributes__ = ["_stacks"]  # the stacked distance-projection rows (host-side scratch)

    def __init__(self, hidden_channels, num_rbf, activation, cutoff_lower, cutoff_upper, trainable_rbf=False,
                 max_z=128, dtype=torch.float32):
        super().__init__()
        self.hidden_channels = hidden_channels
        self.distance_proj1 = nn.Linear(num_rbf, hidden_channels, dtype=dtype)
        self.distance_proj2 = nn.Linear(num_rbf, hidden_channels, dtype=dtype)
        self.distance_proj3 = nn.Linear(num_rbf, hidden_channels, dtype=dtype)
        self.cutoff = CosineCutoff(cutoff_lower, cutoff_upper)
        self.max_z = max_z
        self.emb = nn.Embedding(max_z, hidden_channels, dtype=dtype)
        self.emb2 = nn.Linear(2 * hidden_channels, hidden_channels, dtype=dtype)
        self.act = activation()
        self.linears_tensor = nn.ModuleList()
        for _ in range(3):
            self.linears_tensor.append(nn.Linear(hidden_channels, hidden_channels, bias=False))
        self.linears_scalar = nn.ModuleList()
        self.linears_scalar.append(nn.Linear(hidden_channels, 2 * hidden_channels, bias=True, dtype=dtype))
        self.linears_scalar.append(nn.Linear(2 * hidden_channels, 3 * hidden_channels, bias=True, dtype=dtype))
        self.init_norm = nn.LayerNorm(hidden_channels, dtype=dtype)
        self.reset_parameters()

    def reset_parameters(self):
        self.distance_proj1.reset_parameters()
        self.distance_proj2.reset_parameters()
        self.distance_proj3.reset_parameters()
        self.emb.reset_parameters()
        self.emb2.reset_parameters()
        for linear in self.linears_tensor:
            linear.reset_parameters()
        for linear in self.linears_scalar:
            linear.reset_parameters()
        self.init_norm.reset_parameters()

    def script_forward(self, z: Tensor, row_ptr: Tensor, src: Tensor, dst: Tensor, edge_attr: Tensor, C: Tensor,
                       u: Tensor, m: float) -> Tensor:
        """TorchScript path: reference tensornet.py:295-326 (edge aggregation = tmdnet::tn_embed)."""
        H = self.hidden_channels
        W = torch.nn.functional.linear(
            edge_attr, torch.cat([self.distance_proj1.weight, self.distance_proj2.weight, self.distance_proj3.weight]),
            torch.cat([self.distance_proj1.bias, self.distance_proj2.bias, self.distance_proj3.bias]))
        Z = self.emb(z)
        P = torch.nn.functional.linear(Z, self.emb2.weight[:, :H], self.emb2.bias)
        Q = torch.nn.functional.linear(Z, self.emb2.weight[:, H:])
        Ec = torch.ops.tmdnet.tn_embed(P, Q, W, C, u, row_ptr, src, dst, m)
        norm = self.init_norm(_s_tnorm(_s_full9(Ec)))
        Ec = _s_mix3(Ec, self.linears_tensor[0].weight, self.linears_tensor[1].weight, self.linears_tensor[2].weight)
        for linear_scalar in self.linears_scalar:
            norm = self.act(linear_scalar(norm))
        f = norm.view(norm.shape[0], -1, 3)
        scale = torch.stack([f[..., 0], f[..., 1], f[..., 1], f[..., 1], f[..., 2], f[..., 2], f[..., 2],
                             f[..., 2], f[..., 2]], dim=0)
        return _s_full9(Ec * scale)

    def forward(self, z: Tensor, edge_index: Tensor, edge_weight: Tensor, edge_vec_norm: Tensor,
                edge_attr: Tensor) -> Tensor:
        if torch.jit.is_scripting():
            raise RuntimeError("scripted TensorEmbedding: use script_forward (CSR graph)")
        graph, perm = _check_symmetric_graph(edge_index, z.shape[0])
        if perm is not None:
            edge_weight, edge_vec_norm, edge_attr = edge_weight[perm], edge_vec_norm[perm], edge_attr[perm]
        C = graph.cutoff if (perm is None and graph.cutoff is not None) else self.cutoff(edge_weight)
        H = self.hidden_channels
        # the Linears as kernels.linear: the hand-written MFMA GEMMs (tmdnet_gemm_f32 forward and input
        # gradient, the grouped TN kernel for weight gradients) instead of the library's small-GEMM tiles
        # the three distance projections as row blocks of one weight / bias (no per-step concatenation)
        stacks = self.__dict__.setdefault("_stacks", {})
        dp = (self.distance_proj1, self.distance_proj2, self.distance_proj3)
        W = kernels.linear(edge_attr, kernels.stacked_rows(stacks, "w", [m.weight for m in dp]),
                           kernels.stacked_rows(stacks, "b", [m.bias for m in dp]))
        Z, = kernels.embedding(z, self.emb.weight)
        P = kernels.linear(Z, self.emb2.weight[:, :H], self.emb2.bias)
        Q = kernels.linear(Z, self.emb2.weight[:, H:])
        Ec = kernels.tn_embed(P, Q, W, C, edge_vec_norm, graph)  # compact [9, N, H]: I | A | S rows
        ln = self.init_norm
        en, Ec = tn_node.enorm(Ec, fanout=True)  # (Ec's second consumer's gradient joins in the ENORM bwd)
        norm = kernels.layer_norm(en, ln.weight, ln.bias, ln.eps)
        lt = self.linears_tensor
        Ec = tn_node.mix3(Ec, lt[0].weight, lt[1].weight, lt[2].weight)
        ls = self.linears_scalar  # Linear + act stack, the activations in the GEMM epilogues
        norm = kernels.mlp_act(norm, [m.weight for m in ls], [m.bias for m in ls], self.act)
        # new_radial_tensor(I, A, S, norm[..., 0], norm[..., 1], norm[..., 2]) and I + A + S
        return tn_node.eout(Ec, norm)


class Interaction(nn.Module):
    def __init__(self, num_rbf, hidden_channels, activation, cutoff_lower, cutoff_upper,
                 equivariance_invariance_group, dtype=torch.float32):
        super().__init__()
        self.num_rbf = num_rbf
        self.hidden_channels = hidden_channels
        self.cutoff = CosineCutoff(cutoff_lower, cutoff_upper)
        self.linears_scalar = nn.ModuleList()
        self.linears_scalar.append(nn.Linear(num_rbf, hidden_channels, bias=True, dtype=dtype))
        self.linears_scalar.append(nn.Linear(hidden_channels, 2 * hidden_channels, bias=True, dtype=dtype))
        self.linears_scalar.append(nn.Linear(2 * hidden_channels, 3 * hidden_channels, bias=True, dtype=dtype))
        self.linears_tensor = nn.ModuleList()
        for _ in range(6):
            self.linears_tensor.append(nn.Linear(hidden_channels, hidden_channels, bias=False))
        self.act = activation()
        self.equivariance_invariance_group = equivariance_invariance_group
        self.reset_parameters()

    def reset_parameters(self):
        for linear in self.linears_scalar:
            linear.reset_parameters()
        for linear in self.linears_tensor:
            linear.reset_parameters()

    def script_forward(self, X: Tensor, row_ptr: Tensor, src: Tensor, dst: Tensor, edge_attr: Tensor, C: Tensor,
                       m: float) -> Tensor:
        """TorchScript path: reference tensornet.py:378-410 (message passing = tmdnet::tn_message)."""
        for linear_scalar in self.linears_scalar:
            edge_attr = self.act(linear_scalar(edge_attr))
        edge_attr = edge_attr * C.view(-1, 1)
        lt = self.linears_tensor
        Xn = X / (_s_tnorm(X) + 1)[..., None, None]
        Yc = _s_mix3(_s_decomp9(Xn), lt[0].weight, lt[1].weight, lt[2].weight)
        msg = torch.ops.tmdnet.tn_message(edge_attr, Yc, row_ptr, src, dst, m)
        Y, M = _s_full9(Yc), _s_full9(msg)
        if self.equivariance_invariance_group == "O(3)":
            Z = _s_mm33(M, Y) + _s_mm33(Y, M)
        else:
            Z = 2 * _s_mm33(Y, M)
        Dc = _s_mix3(_s_decomp9(Z) / (_s_tnorm(Z) + 1), lt[3].weight, lt[4].weight, lt[5].weight)
        D = _s_full9(Dc)
        return Xn + D + _s_mm33(D, D)

    def forward(self, X: Tensor, edge_index: Tensor, edge_weight: Tensor, edge_attr: Tensor) -> Tensor:
        if torch.jit.is_scripting():
            raise RuntimeError("scripted Interaction: use script_forward (CSR graph)")
        graph, perm = _check_symmetric_graph(edge_index, X.shape[0])
        if perm is not None:
            edge_weight, edge_attr = edge_weight[perm], edge_attr[perm]
        C = graph.cutoff if (perm is None and graph.cutoff is not None) else self.cutoff(edge_weight)
        ls = self.linears_scalar  # act(Linear) x 3, the last times C (reference 381-385), one launch per layer
        pairs = None
        if (PAIRS and perm is None and X.is_cuda and graph.n_edges >= PAIR_MIN_EDGES and graph.symmetric
                and graph.transpose is not None):
            # one MLP row per edge pair (the factors depend on |r| only): gather the pairs' rbf / cutoff rows
            pairs = kernels.pair_index(graph)
            pe = getattr(graph, "_pair_edge_long", None)
            if pe is None:
                pe = graph._pair_edge_long = pairs[1].long()
            edge_attr, C = edge_attr.index_select(0, pe), C.index_select(0, pe)
        edge_attr = kernels.mlp_act(edge_attr, [m.weight for m in ls], [m.bias for m in ls], self.act, C)
        lt = self.linears_tensor
        # X / (|X|^2 + 1), decompose, three channel mixes -> Y as compact [9, N, H] (I | A | S rows)
        # (the fan-out aliases let X's and Y's second consumers' gradients join inside the PRE / message
        # backward kernels instead of separate autograd add launches)
        Xp, X = tn_node.pre(X, fanout=True)
        Yc = tn_node.mix3(Xp, lt[0].weight, lt[1].weight, lt[2].weight)
        msg, Yc = kernels.tn_message(edge_attr, Yc, graph, fanout=True, pairs=pairs)
        # decompose(msg Y + Y msg) (O(3)) or decompose(2 Y msg) (SO(3)), / (|.|^2 + 1), three mixes
        Dc = tn_node.mix3(tn_node.post(Yc, msg, self.equivariance_invariance_group),
                          lt[3].weight, lt[4].weight, lt[5].weight)
        return tn_node.resid(X, Dc)  # X / (|X|^2 + 1) + dX + dX dX (X was reassigned, :391)
