"""Equivariant Transformer (mirror of reference ``torchmdnet/models/torchmd_et.py``).

Same constructor arguments, module tree, parameter names and initialisation order as the reference
(torchmd_et.py:14-270), so ``create_model`` + ``torch.manual_seed`` reproduce reference weights and
reference checkpoints load.  The per-edge work runs in HIP kernels:
  * neighbour list: CSR EdgeGraph from ``tmdnet_nl_build`` (one build per forward);
  * RBF + cosine cutoff + unit vectors: one fused kernel (``tmdnet_edge_geom_*``), the cutoff is
    computed once and shared by every layer (all layers use the same CosineCutoff(cl, cu));
  * message + aggregation: ``tmdnet_et_message_fwd/bwd`` (wave per destination, no atomics).
The dense node/edge projections (LayerNorm, q/k/v/o/vec, dk/dv) are GEMMs (rocBLAS/hipBLASLt via
torch, MFMA) whose outputs feed the kernels without reshuffling.
"""
import os
from typing import List, Optional, Tuple

import torch
from torch import Tensor, nn

from .. import et_stack as et_stack_mod
from .. import kernels
from ..et_stack import et_stack
from .utils import (CosineCutoff, NeighborEmbedding, OptimizedDistance, act_class_mapping, as_graph,
                    rbf_class_mapping)

# large systems: the neighbour embedding's distance_proj formed inside its aggregation kernel
# (kernels.nbr_embed_fused; same size threshold as the fused layer stack).  TMDNET_NE_FUSED=0: rows (A/B)
NE_FUSED = os.environ.get("TMDNET_NE_FUSED", "1") != "0"
# eval mode, eager, below the fused-projection scale: the interaction layers as the C++ ``tmdnet::et_stack``
# operator (the scripted path's; same kernels, differentiable to any order) instead of the Python
# _ETStack / _ETStackBwd, whose launch orchestration costs ~2 ms of host time per C2 evaluation.  Training
# (train mode: the force-loss second order is hand-written on the Python side) and HIP-graph capture keep
# the Python stack.  C2 eval 2.84 -> 2.17 ms eager; energies / forces equal to the Python stack's to 1e-7.
# The operator caches nothing: its stacked weights are views of the parameters' own storage (stacked here
# before every call, et_stack.stack_parameters), so optimizer steps of any kind and ``p.data`` writes are
# seen by the next evaluation.  TMDNET_ET_CPP_EAGER=0 keeps the Python stack everywhere.
CPP_EAGER = os.environ.get("TMDNET_ET_CPP_EAGER", "1") != "0"


class TorchMD_ET(nn.Module):
    r"""The TorchMD equivariant Transformer architecture (arXiv:2202.02541)."""

    def __init__(self, hidden_channels=128, num_layers=6, num_rbf=50, rbf_type="expnorm",
                 trainable_rbf=True, activation="silu", attn_activation="silu",
                 neighbor_embedding=True, num_heads=8, distance_influence="both", cutoff_lower=0.0,
                 cutoff_upper=5.0, max_z=100, max_num_neighbors=32, dtype=torch.float32):
        super().__init__()
        assert distance_influence in ["keys", "values", "both", "none"]
        assert rbf_type in rbf_class_mapping, (
            f'Unknown RBF type "{rbf_type}". Choose from {", ".join(rbf_class_mapping.keys())}.')
        assert activation in act_class_mapping, (
            f'Unknown activation function "{activation}". Choose from {", ".join(act_class_mapping.keys())}.')
        assert attn_activation in act_class_mapping, (
            f'Unknown attention activation function "{attn_activation}". '
            f'Choose from {", ".join(act_class_mapping.keys())}.')

        self.hidden_channels = hidden_channels
        self.num_layers = num_layers
        self.num_rbf = num_rbf
        self.rbf_type = rbf_type
        self.trainable_rbf = trainable_rbf
        self.activation = activation
        self.attn_activation = attn_activation
        self.neighbor_embedding = neighbor_embedding
        self.num_heads = num_heads
        self.distance_influence = distance_influence
        self.cutoff_lower = cutoff_lower
        self.cutoff_upper = cutoff_upper
        self.max_z = max_z
        self.dtype = dtype

        act_class = act_class_mapping[activation]

        self.embedding = nn.Embedding(self.max_z, hidden_channels, dtype=dtype)
        self.distance = OptimizedDistance(cutoff_lower, cutoff_upper, max_num_pairs=-max_num_neighbors,
                                          return_vecs=True, loop=True, long_edge_index=True)
        self.distance.pair_rows = True  # the layer stack's pair-shared dk/dv rows (et_stack.PAIR_ROWS)
        self.distance_expansion = rbf_class_mapping[rbf_type](cutoff_lower, cutoff_upper, num_rbf, trainable_rbf)
        self.neighbor_embedding = (
            NeighborEmbedding(hidden_channels, num_rbf, cutoff_lower, cutoff_upper, self.max_z, dtype).jittable()
            if neighbor_embedding else None)

        self.attention_layers = nn.ModuleList()
        for _ in range(num_layers):
            layer = EquivariantMultiHeadAttention(hidden_channels, num_rbf, distance_influence, num_heads,
                                                  act_class, attn_activation, cutoff_lower, cutoff_upper,
                                                  dtype).jittable()
            self.attention_layers.append(layer)

        self.out_norm = nn.LayerNorm(hidden_channels, dtype=dtype)
        self.reorder_atoms = True
        self.fused_stack = True
        self.reset_parameters()

    def reset_parameters(self):
        self.embedding.reset_parameters()
        self.distance_expansion.reset_parameters()
        if self.neighbor_embedding is not None:
            self.neighbor_embedding.reset_parameters()
        for attn in self.attention_layers:
            attn.reset_parameters()
        self.out_norm.reset_parameters()

    def __prepare_scriptable__(self):
        for attn in self.attention_layers:
            attn._check_supported()
        if len(self.attention_layers) > 0:
            # the scripted operators take the stacked weights as views of the parameters (torch_ops.cpp pack_stack)
            et_stack_mod.stack_parameters(self.attention_layers)
        return self

    def forward(self, z: Tensor, pos: Tensor, batch: Tensor, q: Optional[Tensor] = None,
                s: Optional[Tensor] = None) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor]:
        if torch.jit.is_scripting():
            x, vec = self._forward_script(z, pos, batch)
            return x, vec, z, pos, batch
        perm = None
        if self.reorder_atoms and z.shape[0] >= kernels.REORDER_MIN_ATOMS:
            # large systems: compute in a spatially coherent atom numbering (edge-kernel locality);
            # outputs are returned in the caller's order, forces flow back through the gather.
            perm = kernels.spatial_permutation(pos, batch, self.cutoff_upper,
                                               self.distance.box if self.distance.use_periodic else None)
            inv = torch.empty_like(perm)
            inv[perm] = torch.arange(perm.numel(), device=perm.device)
            x, vec = self._forward(z[perm], pos.index_select(0, perm), batch[perm])
            return x[inv], vec[inv], z, pos, batch
        x, vec = self._forward(z, pos, batch)
        return x, vec, z, pos, batch

    def _forward_script(self, z: Tensor, pos: Tensor, batch: Tensor) -> Tuple[Tensor, Tensor]:
        """TorchScript path (torch.jit.script(model)) over the dispatcher operators of
        libtmdnet_torch.so -- neighbour list, edge geometry and neighbour embedding are the HIP kernels
        with C++ autograd; the interaction layers (fp32, fixed RBF basis) run as ONE ``tmdnet::et_stack``
        operator with the eager stack's fused launches and dr-mode force backward (differentiable to any
        order: parameter gradients and higher orders by recompute).  fp64 or a trainable basis: the
        reference layer loop (torchmd_et.py:160-190) over ``tmdnet::et_message`` with ATen node GEMMs."""
        x = self.embedding(z)
        d = self.distance
        row_ptr, src, dst, tr, deltas, dist, num_pairs = torch.ops.tmdnet.neighbor_graph(
            pos, batch, d.box, d.use_periodic, float(d.cutoff_lower), float(d.cutoff_upper),
            d._max_pairs(pos.shape[0]), d.loop, d.strategy, d.check_errors, -1)
        de = self.distance_expansion
        mu, beta = de.kernel_params()
        trainable = self.trainable_rbf and torch.is_grad_enabled()
        f, C, u = torch.ops.tmdnet.edge_geometry(deltas, dist, src, dst, mu, beta, float(self.cutoff_lower),
                                                 float(self.cutoff_upper), de.rbf_type, not trainable)
        if trainable:  # trainable basis: differentiable ATen features (the parameters need gradients)
            f = de(dist)
        ne = self.neighbor_embedding
        if ne is not None:
            x = ne.script_forward(z, x, row_ptr, src, dst, f, C)
        if self.fused_stack and not trainable and x.dtype == torch.float32 and len(self.attention_layers) > 0:
            # every layer + out_norm as ONE operator (tmdnet::et_stack): the eager stack's fused launches
            # and its dr-mode force backward (et_stack.py), f delivered as rbf(dist)
            params: List[Tensor] = []
            hk = False
            hv = False
            acts = 0
            for attn in self.attention_layers:
                params += attn.stack_params()
                hk = attn.dk_proj is not None
                hv = attn.dv_proj is not None
                acts = attn.act_flags
            on = self.out_norm
            fuse_norm = on.elementwise_affine and on.eps == 1e-5
            if fuse_norm:
                params += [on.weight, on.bias]
            x, vec = torch.ops.tmdnet.et_stack(x, f, dist, C, u, mu, beta, row_ptr, src, dst, float(self.cutoff_lower),
                                               float(self.cutoff_upper), de.rbf_type, self.num_heads, hk, hv,
                                               fuse_norm, params, acts)
            if not fuse_norm:
                x = on(x)
            return x, vec
        vec = torch.zeros(x.size(0), 3, x.size(1), device=x.device, dtype=x.dtype)
        for attn in self.attention_layers:
            dx, dvec = attn.script_forward(x, vec, row_ptr, src, dst, f, C, u)
            x = x + dx
            vec = vec + dvec
        x = self.out_norm(x)
        return x, vec

    def fused_energy_forces(self, z: Tensor, pos: Tensor, batch: Tensor, head: List[Tensor], std: Tensor,
                            mean: Tensor) -> Tuple[Tensor, Tensor]:
        """(y, neg_dy) of TorchMD_Net(this model, EquivariantScalar head) as ONE operator,
        tmdnet::et_energy_forces (TorchMD_Net.fused_eval: TorchScript inference in eval mode)."""
        d = self.distance
        de = self.distance_expansion
        mu, beta = de.kernel_params()
        params: List[Tensor] = []
        hk = False
        hv = False
        acts = 0
        for attn in self.attention_layers:
            params += attn.stack_params()
            hk = attn.dk_proj is not None
            hv = attn.dv_proj is not None
            acts = attn.act_flags
        params += [self.out_norm.weight, self.out_norm.bias]
        nb_emb: Optional[Tensor] = None
        nb_dw: Optional[Tensor] = None
        nb_db: Optional[Tensor] = None
        nb_cw: Optional[Tensor] = None
        nb_cb: Optional[Tensor] = None
        ne = self.neighbor_embedding
        if ne is not None:
            nb_emb = ne.embedding.weight
            nb_dw = ne.distance_proj.weight
            nb_db = ne.distance_proj.bias
            nb_cw = ne.combine.weight
            nb_cb = ne.combine.bias
        return torch.ops.tmdnet.et_energy_forces(
            z, pos, batch, d.box, d.use_periodic, float(d.cutoff_lower), float(d.cutoff_upper),
            d._max_pairs(pos.shape[0]), d.loop, d.strategy, d.check_errors, self.embedding.weight, nb_emb, nb_dw,
            nb_db, nb_cw, nb_cb, mu, beta, de.rbf_type, self.num_heads, hk, hv, True, params, acts, head, std, mean)

    def _forward(self, z: Tensor, pos: Tensor, batch: Tensor):
        ne = self.neighbor_embedding
        x_ne = None
        if z.is_cuda and ne is not None:  # both tables' lookups (and gradients) in one node
            x, x_ne = kernels.embedding(z, self.embedding.weight, ne.embedding.weight)
        elif z.is_cuda:
            x, = kernels.embedding(z, self.embedding.weight)
        else:
            x = self.embedding(z)
        graph = self.distance.graph(pos, batch)
        f_pairs = fdp_pairs = None
        ne_fused = None
        edge_attr_s = C_s = None  # the layer stack's aliases of the rbf / cutoff rows
        de = self.distance_expansion
        if self.trainable_rbf and torch.is_grad_enabled():
            # trainable basis: parameters need gradients -> differentiable torch basis on the GPU
            edge_attr = de(graph.distances)
            _, C, d_ij = kernels.edge_geometry(graph, *de.kernel_params(), self.cutoff_lower,
                                               self.cutoff_upper, de.rbf_type, want=(False, True, True))
        else:
            pairs = getattr(graph, "_pairs", None)  # numbered by the neighbour build (sorted rows)
            stack = self.fused_stack and len(self.attention_layers) > 0
            # (no pair rows where the stack forms the projection in-kernel: at C5 they are 350 MB unread)
            fep_scale = graph.n_edges >= et_stack_mod.FEP_MIN_EDGES and et_stack_mod.FEP not in ("0", "off")
            rows = pairs[1] if (pairs is not None and stack and not fep_scale) else None
            ne = self.neighbor_embedding
            if (ne is not None and z.is_cuda and NE_FUSED and graph.n_edges >= et_stack_mod.FEP_MIN_EDGES
                    and et_stack_mod.FEP not in ("0", "off")
                    and kernels.nbr_fused_supported(graph, self.hidden_channels, self.num_rbf, pos.dtype)):
                # large systems: distance_proj formed inside the aggregation kernel from r (no rbf or
                # projection rows for the neighbour embedding; dr-mode force backward)
                mu, beta = de.kernel_params()
                ne_fused = ((mu.detach(), beta.detach(), float(self.cutoff_lower), float(self.cutoff_upper),
                             int(de.rbf_type)), de)
            # rbf and cutoff rows read by the neighbour embedding AND the layer stack: one alias each, their
            # gradients summed in the geometry backward kernel (no autograd add launch)
            fan = (1, 1)
            if stack and ne is not None:
                fan = (1, 2) if ne_fused is not None else (2, 2)
            # a force pass to follow (pos differentiated): the pair rows' d rbf / d r from the same launch
            drows = rows is not None and pos.requires_grad and torch.is_grad_enabled()
            geo = kernels.edge_geometry(graph, *de.kernel_params(), self.cutoff_lower, self.cutoff_upper,
                                        de.rbf_type, rows=rows, fan=fan, drows=drows)
            edge_attr, C, d_ij = geo[:3]
            f_pairs = geo[3] if rows is not None else None
            fdp_pairs = geo[4] if drows else None
            if fan == (2, 2):
                (edge_attr, edge_attr_s), (C, C_s) = edge_attr, C
            elif fan == (1, 2):
                (edge_attr_s,), (C, C_s) = edge_attr, C
                edge_attr = None
        if edge_attr_s is None:
            edge_attr_s, C_s = edge_attr, C
        graph.cutoff = C_s
        if self.neighbor_embedding is not None:
            if ne_fused is not None:
                x = self.neighbor_embedding.fused_forward(z, x, graph, graph.distances, C, x_ne, *ne_fused)
            else:
                x = self.neighbor_embedding(z, x, graph, graph.distances, edge_attr, cutoff=C, x_emb=x_ne)
        if self.fused_stack and len(self.attention_layers) > 0:
            # all layers as one autograd node (et_stack.py): fused GEMMs, HIP epilogue, hand-scheduled
            # backward; same math as the loop below
            rbf = None
            if not (self.trainable_rbf and torch.is_grad_enabled()):  # fixed basis: f = rbf(r)
                # (r's alias: the stack's g_r joins the geometry's in the neighbour backward kernel)
                r_s = getattr(graph, "distances_alias", None)
                rbf = (graph.distances if r_s is None else r_s, *de.kernel_params(), self.cutoff_lower,
                       self.cutoff_upper, de.rbf_type)
            on = self.out_norm
            fuse_norm = on.elementwise_affine and on.eps == 1e-5
            if (CPP_EAGER and rbf is not None and not self.training and x.is_cuda and x.dtype == torch.float32
                    and graph.symmetric and not graph.static and graph.n_edges < et_stack_mod.FEP_MIN_EDGES
                    and not torch.cuda.is_current_stream_capturing()):
                x, vec = self._stack_op(x, graph, edge_attr_s, C_s, d_ij, rbf, fuse_norm)
            else:
                x, vec = et_stack(self.attention_layers, x, graph, edge_attr_s, C_s, d_ij, rbf=rbf,
                                  out_norm=on if fuse_norm else None, f_pairs=f_pairs, fdp_pairs=fdp_pairs)
            return (x if fuse_norm else on(x)), vec
        vec = torch.zeros(x.size(0), 3, x.size(1), device=x.device, dtype=x.dtype)
        for attn in self.attention_layers:
            dx, dvec = attn(x, vec, graph, graph.distances, edge_attr, d_ij)
            x = x + dx
            vec = vec + dvec
        x = self.out_norm(x)
        return x, vec

    @torch.jit.unused
    def _stack_op(self, x, graph, f, C, u, rbf, fuse_norm):
        """The interaction layers as ``tmdnet::et_stack`` (see CPP_EAGER)."""
        from .. import _native
        _native.load_torch_ops()
        et_stack_mod.stack_parameters(self.attention_layers)  # (views, not copies: see CPP_EAGER)
        r, mu, beta, cl, cu, rbf_type = rbf
        params = []
        hk = hv = False
        acts = 0
        for attn in self.attention_layers:
            params += attn.stack_params()
            hk = attn.dk_proj is not None
            hv = attn.dv_proj is not None
            acts = attn.act_flags
        if fuse_norm:
            params += [self.out_norm.weight, self.out_norm.bias]
        return torch.ops.tmdnet.et_stack(x, f, r, C, u, mu, beta, graph.row_ptr, graph.src, graph.dst, float(cl),
                                         float(cu), rbf_type, self.num_heads, hk, hv, fuse_norm, params, acts)

    def __repr__(self):
        return (f"{self.__class__.__name__}(hidden_channels={self.hidden_channels}, "
                f"num_layers={self.num_layers}, num_rbf={self.num_rbf}, rbf_type={self.rbf_type}, "
                f"trainable_rbf={self.trainable_rbf}, activation={self.activation}, "
                f"attn_activation={self.attn_activation}, neighbor_embedding={self.neighbor_embedding}, "
                f"num_heads={self.num_heads}, distance_influence={self.distance_influence}, "
                f"cutoff_lower={self.cutoff_lower}, cutoff_upper={self.cutoff_upper}), dtype={self.dtype}")


class EquivariantMultiHeadAttention(nn.Module):
    """Reference torchmd_et.py:208-352.  forward(x, vec, edge_index, r_ij, f_ij, d_ij) -> (dx, dvec)."""

    def __init__(self, hidden_channels, num_rbf, distance_influence, num_heads, activation,
                 attn_activation, cutoff_lower, cutoff_upper, dtype=torch.float32):
        super().__init__()
        assert hidden_channels % num_heads == 0, (
            f"The number of hidden channels ({hidden_channels}) must be evenly divisible by the number "
            f"of attention heads ({num_heads})")
        self.distance_influence = distance_influence
        self.num_heads = num_heads
        self.hidden_channels = hidden_channels
        self.head_dim = hidden_channels // num_heads
        self.layernorm = nn.LayerNorm(hidden_channels, dtype=dtype)
        self.act = activation()
        self.attn_activation = act_class_mapping[attn_activation]()
        # both activations as the edge kernels' codes (SiLU / ShiftedSoftplus / Tanh / Sigmoid)
        self.act_flags = kernels.et_act_flags(kernels.act_code(self.act), kernels.act_code(self.attn_activation))
        self.cutoff = CosineCutoff(cutoff_lower, cutoff_upper)

        self.q_proj = nn.Linear(hidden_channels, hidden_channels, dtype=dtype)
        self.k_proj = nn.Linear(hidden_channels, hidden_channels, dtype=dtype)
        self.v_proj = nn.Linear(hidden_channels, hidden_channels * 3, dtype=dtype)
        self.o_proj = nn.Linear(hidden_channels, hidden_channels * 3, dtype=dtype)
        self.vec_proj = nn.Linear(hidden_channels, hidden_channels * 3, bias=False, dtype=dtype)
        self.dk_proj = None
        if distance_influence in ["keys", "both"]:
            self.dk_proj = nn.Linear(num_rbf, hidden_channels, dtype=dtype)
        self.dv_proj = None
        if distance_influence in ["values", "both"]:
            self.dv_proj = nn.Linear(num_rbf, hidden_channels * 3, dtype=dtype)
        self._stacked = None  # et_stack.LayerWeights: q/k/v and dk/dv parameters as stacked views
        self.reset_parameters()

    def jittable(self):
        return self

    def reset_parameters(self):
        self.layernorm.reset_parameters()
        nn.init.xavier_uniform_(self.q_proj.weight)
        self.q_proj.bias.data.fill_(0)
        nn.init.xavier_uniform_(self.k_proj.weight)
        self.k_proj.bias.data.fill_(0)
        nn.init.xavier_uniform_(self.v_proj.weight)
        self.v_proj.bias.data.fill_(0)
        nn.init.xavier_uniform_(self.o_proj.weight)
        self.o_proj.bias.data.fill_(0)
        nn.init.xavier_uniform_(self.vec_proj.weight)
        if self.dk_proj:
            nn.init.xavier_uniform_(self.dk_proj.weight)
            self.dk_proj.bias.data.fill_(0)
        if self.dv_proj:
            nn.init.xavier_uniform_(self.dv_proj.weight)
            self.dv_proj.bias.data.fill_(0)

    def _check_supported(self):
        """Re-derive the kernels' activation codes (the modules may have been replaced after
        construction); raises NotImplementedError outside the reference's act_class_mapping."""
        self.act_flags = kernels.et_act_flags(kernels.act_code(self.act), kernels.act_code(self.attn_activation))

    def stack_params(self) -> List[Tensor]:
        """This layer's parameters in tmdnet::et_stack's order (et_stack.layer_params)."""
        ps = [self.layernorm.weight, self.layernorm.bias, self.q_proj.weight, self.q_proj.bias,
              self.k_proj.weight, self.k_proj.bias, self.v_proj.weight, self.v_proj.bias,
              self.vec_proj.weight, self.o_proj.weight, self.o_proj.bias]
        if self.dk_proj is not None:
            ps += [self.dk_proj.weight, self.dk_proj.bias]
        if self.dv_proj is not None:
            ps += [self.dv_proj.weight, self.dv_proj.bias]
        return ps

    def script_forward(self, x: Tensor, vec: Tensor, row_ptr: Tensor, src: Tensor, dst: Tensor, f_ij: Tensor,
                       C: Tensor, d_ij: Tensor) -> Tuple[Tensor, Tensor]:
        """TorchScript path: reference torchmd_et.py:293-321 with message + aggregate as
        ``tmdnet::et_message`` (HIP, C++ autograd)."""
        x = self.layernorm(x)
        q = self.q_proj(x)
        k = self.k_proj(x)
        v = self.v_proj(x)
        vec1, vec2, vec3 = torch.split(self.vec_proj(vec), self.hidden_channels, dim=-1)
        vec_dot = (vec1 * vec2).sum(dim=1)
        pk: Optional[Tensor] = None
        pv: Optional[Tensor] = None
        if self.dk_proj is not None:
            pk = self.dk_proj(f_ij)
        if self.dv_proj is not None:
            pv = self.dv_proj(f_ij)
        xa, veca = torch.ops.tmdnet.et_message(q, k, v, vec, pk, pv, C, d_ij, row_ptr, src, dst, self.num_heads,
                                               self.act_flags)
        o1, o2, o3 = torch.split(self.o_proj(xa), self.hidden_channels, dim=1)
        return vec_dot * o2 + o3, vec3 * o1.unsqueeze(1) + veca

    def forward(self, x: Tensor, vec: Tensor, edge_index: Tensor, r_ij: Tensor, f_ij: Tensor,
                d_ij: Tensor) -> Tuple[Tensor, Tensor]:
        if torch.jit.is_scripting():
            raise RuntimeError("scripted EquivariantMultiHeadAttention: use script_forward (CSR graph)")
        self._check_supported()
        graph, perm = as_graph(edge_index, x.shape[0])
        if perm is not None:
            r_ij, f_ij, d_ij = r_ij[perm], f_ij[perm], d_ij[perm]
        C = graph.cutoff if (perm is None and graph.cutoff is not None) else self.cutoff(r_ij)
        x = self.layernorm(x)
        q = self.q_proj(x)
        k = self.k_proj(x)
        v = self.v_proj(x)
        vec1, vec2, vec3 = torch.split(self.vec_proj(vec), self.hidden_channels, dim=-1)
        vec_dot = (vec1 * vec2).sum(dim=1)
        pk = self.dk_proj(f_ij) if self.dk_proj is not None else None
        pv = self.dv_proj(f_ij) if self.dv_proj is not None else None
        xa, veca = kernels.et_message(q, k, v, vec, pk, pv, C, d_ij, graph, self.num_heads, self.act_flags)
        o1, o2, o3 = torch.split(self.o_proj(xa), self.hidden_channels, dim=1)
        dx = vec_dot * o2 + o3
        dvec = vec3 * o1.unsqueeze(1) + veca
        return dx, dvec
