"""Output heads (mirror of reference ``torchmdnet/models/output_modules.py``).

Node-level and tiny (H -> H/2 -> 1 per atom); they run as PyTorch GPU ops.  ``reduce`` sums atoms
into molecules with ``index_add`` (the reference uses torch_scatter, output_modules.py:27-43).
"""
from abc import ABCMeta, abstractmethod
from typing import List, Optional

import torch
from torch import nn

from .. import kernels
from .utils import GatedEquivariantBlock, act_class_mapping, check_stream_capturing
from ..utils import atomic_masses

__all__ = ["Scalar", "DipoleMoment", "ElectronicSpatialExtent"]


def scatter(src, index, dim=0, dim_size=None, reduce="sum"):
    """Segment reduction over dim 0 (sum/add/mean), torch_scatter 2.1.1 semantics for this use."""
    if dim_size is None:
        dim_size = int(index.max().item()) + 1
    out = torch.zeros((dim_size,) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
    out = out.index_add(0, index, src)
    if reduce in ("sum", "add"):
        return out
    if reduce == "mean":
        cnt = torch.zeros(dim_size, dtype=src.dtype, device=src.device).index_add(
            0, index, torch.ones_like(index, dtype=src.dtype))
        return out / cnt.clamp(min=1).view(-1, *([1] * (src.dim() - 1)))
    raise NotImplementedError(f"reduce_op {reduce}")


class OutputModel(nn.Module, metaclass=ABCMeta):
    def __init__(self, allow_prior_model, reduce_op):
        super().__init__()
        self.allow_prior_model = allow_prior_model
        self.reduce_op = reduce_op
        self.dim_size = 0
        self.dim_size_hint = -1  # the molecule count, read back early by TorchMD_Net.forward (-1: none)

    def reset_parameters(self):
        pass

    @abstractmethod
    def pre_reduce(self, x, v, z, pos, batch):
        return

    def _dim_size(self, x, batch):
        is_capturing = x.is_cuda and check_stream_capturing()
        if not x.is_cuda or not is_capturing:
            if self.dim_size_hint >= 0:  # (read back before the forward was enqueued: no wait here)
                self.dim_size, self.dim_size_hint = self.dim_size_hint, -1
            else:
                self.dim_size = int(batch.max().item() + 1)
        if is_capturing:
            assert self.dim_size > 0, "Warming up is needed before capturing the model into a CUDA graph"
        return self.dim_size

    def reduce(self, x, batch):
        if torch.jit.is_scripting():  # reference output_modules.py:27-43 (scatter sum / mean)
            dim_size = int(batch.max().item()) + 1
            out = torch.zeros([dim_size] + x.shape[1:], dtype=x.dtype, device=x.device).index_add(0, batch, x)
            if self.reduce_op == "mean":
                cnt = torch.zeros(dim_size, dtype=x.dtype, device=x.device).index_add(
                    0, batch, torch.ones(batch.shape[0], dtype=x.dtype, device=x.device))
                out = out / cnt.clamp(min=1).view([dim_size] + [1] * (x.dim() - 1))
            return out
        return scatter(x, batch, dim=0, dim_size=self._dim_size(x, batch), reduce=self.reduce_op)

    def fused_reduce(self, x, batch, std, mean):
        """``reduce(x * std) + mean`` as one HIP pass (TorchMD_Net.forward without priors), or None
        when this head's reduction is not the plain per-molecule sum."""
        if not (x.is_cuda and self.reduce_op in ("sum", "add") and x.dim() == 2 and x.shape[1] == 1
                and type(self).reduce is OutputModel.reduce and batch.dtype == torch.int64
                and std is not None and mean is not None and std.numel() == 1 and mean.numel() == 1):
            return None
        n_mol = self._dim_size(x, batch)
        if n_mol > kernels.ATOM_SUM_MAX_MOLECULES:
            return None
        return kernels.atom_sum(x, batch, n_mol, std.to(x.dtype), mean.to(x.dtype))

    def post_reduce(self, x):
        return x

    def fused_head_reduce(self, x, v, z, pos, batch, std, mean):
        """``reduce(pre_reduce(x, ...) * std) + mean`` with the head's tail fused into the reduction, or
        None when this head has no such form (TorchMD_Net.forward then runs pre_reduce + fused_reduce)."""
        return None

    def head_params(self) -> List[torch.Tensor]:
        """The fused head kernel's tensors (EquivariantScalar; empty for other heads)."""
        return []


class Scalar(OutputModel):
    def __init__(self, hidden_channels, activation="silu", allow_prior_model=True, reduce_op="sum",
                 dtype=torch.float):
        super().__init__(allow_prior_model=allow_prior_model, reduce_op=reduce_op)
        act_class = act_class_mapping[activation]
        self.output_network = nn.Sequential(
            nn.Linear(hidden_channels, hidden_channels // 2, dtype=dtype),
            act_class(),
            nn.Linear(hidden_channels // 2, 1, dtype=dtype),
        )
        self.reset_parameters()

    def reset_parameters(self):
        nn.init.xavier_uniform_(self.output_network[0].weight)
        self.output_network[0].bias.data.fill_(0)
        nn.init.xavier_uniform_(self.output_network[2].weight)
        self.output_network[2].bias.data.fill_(0)

    def pre_reduce(self, x, v: Optional[torch.Tensor], z, pos, batch):
        if torch.jit.is_scripting():
            return self.output_network(x)
        net = self.output_network
        return net[2](kernels.fused_act(net[1], net[0](x)))

    @torch.jit.unused
    def fused_head_reduce(self, x, v, z, pos, batch, std, mean):
        """Linear + SiLU as one hand GEMM launch (kernels.mlp_act), then the last Linear (H/2 -> 1) fused
        with `x * std`, the per-molecule sum and `+ mean` (kernels.dot_sum): 2 launches (their backward 2)
        instead of two library GEMMs, the activation, the reduction and their backward passes."""
        net = self.output_network
        if not (x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and isinstance(net[1], nn.SiLU)
                and self.reduce_op in ("sum", "add") and batch.dtype == torch.int64 and std is not None
                and mean is not None and std.numel() == 1 and mean.numel() == 1
                and net[0].out_features % 16 == 0 and net[0].in_features % 16 == 0):
            return None
        n_mol = self._dim_size(x, batch)
        if n_mol > kernels.ATOM_SUM_MAX_MOLECULES:
            return None
        h = kernels.mlp_act(x, [net[0].weight], [net[0].bias], net[1])
        return kernels.dot_sum(h, net[2].weight, net[2].bias, batch, n_mol, std.to(x.dtype), mean.to(x.dtype))


class EquivariantScalar(OutputModel):
    def __init__(self, hidden_channels, activation="silu", allow_prior_model=True, reduce_op="sum",
                 dtype=torch.float):
        super().__init__(allow_prior_model=allow_prior_model, reduce_op=reduce_op)
        self.output_network = nn.ModuleList([
            GatedEquivariantBlock(hidden_channels, hidden_channels // 2, activation=activation,
                                  scalar_activation=True, dtype=dtype),
            GatedEquivariantBlock(hidden_channels // 2, 1, activation=activation, dtype=dtype),
        ])
        self.reset_parameters()

    def reset_parameters(self):
        for layer in self.output_network:
            layer.reset_parameters()

    def head_params(self) -> List[torch.Tensor]:
        """The 12 tensors of tmdnet_eq_head_fwd in its order (kernels.eq_head_params)."""
        ps: List[torch.Tensor] = []
        for b in self.output_network:
            ps += [b.vec1_proj.weight, b.vec2_proj.weight, b.update_net[0].weight, b.update_net[0].bias,
                   b.update_net[2].weight, b.update_net[2].bias]
        return ps

    def _gated(self, x, v):
        """(scalar, vector) outputs of the two gated blocks."""
        for block in self.output_network:
            x, v = block(x, v)
        return x, v

    def pre_reduce(self, x, v, z, pos, batch):
        if torch.jit.is_scripting():  # reference output_modules.py:98-103
            for layer in self.output_network:
                x, v = layer(x, v)
            return x + v.sum() * 0
        if x.is_cuda and type(self) is EquivariantScalar and kernels.eq_head_fusable(self.output_network):
            # both gated blocks + the per-atom Jacobian in one HIP kernel (csrc/eq_head.hip); the
            # reference's "+ 0 * v.sum()" only keeps v in the autograd graph and adds nothing
            return kernels.eq_scalar_head(x, v, self.output_network)
        for layer in self.output_network:
            x, v = layer(x, v)
        return x + v.sum() * 0


# ----------------------------------------------------------------------------- secondary heads
# Dipole / spatial-extent / vector heads (interface of reference output_modules.py:117-207: class names and
# the state_dict layout of their networks).  Not on the hot path (SURVEY §8 names only the energy heads); they
# run as plain tensor code.  Shared pieces: the mass-weighted centre of each molecule, and the gated blocks'
# (scalar, vector) output of EquivariantScalar.


def _offsets_from_centre(masses, z, pos, batch):
    """pos minus its molecule's centre of mass, one row per atom."""
    m = masses.index_select(0, z).unsqueeze(1)
    n_mol = int(batch.max()) + 1 if batch.numel() else 0
    acc = pos.new_zeros(n_mol, 4).index_add_(0, batch, torch.cat([pos * m, m], dim=1))
    centre = acc[:, :3] / acc[:, 3:]
    return pos - centre.index_select(0, batch)


class _MassTable(nn.Module):
    """Holds the ``atomic_mass`` buffer (a state_dict key of the reference heads)."""

    def _add_masses(self, dtype):
        self.register_buffer("atomic_mass", torch.as_tensor(atomic_masses, dtype=dtype))


class DipoleMoment(Scalar, _MassTable):
    """Per-atom partial charges q_i from the scalar network; reduces sum_i q_i (r_i - r_com) and returns its norm."""

    def __init__(self, hidden_channels, activation="silu", reduce_op="sum", dtype=torch.float):
        super().__init__(hidden_channels, activation, allow_prior_model=False, reduce_op=reduce_op, dtype=dtype)
        self._add_masses(dtype)

    def pre_reduce(self, x, v: Optional[torch.Tensor], z, pos, batch):
        charges = self.output_network(x)
        return charges * _offsets_from_centre(self.atomic_mass, z, pos, batch)

    def post_reduce(self, x):
        return x.norm(dim=-1, keepdim=True)


class EquivariantDipoleMoment(EquivariantScalar, _MassTable):
    """Charges plus a per-atom dipole vector from the gated blocks: q_i (r_i - r_com) + mu_i, then the norm."""

    def __init__(self, hidden_channels, activation="silu", reduce_op="sum", dtype=torch.float):
        super().__init__(hidden_channels, activation, allow_prior_model=False, reduce_op=reduce_op, dtype=dtype)
        self._add_masses(dtype)

    def pre_reduce(self, x, v, z, pos, batch):
        charges, mu = self._gated(x, v)
        return charges * _offsets_from_centre(self.atomic_mass, z, pos, batch) + mu.squeeze()

    def post_reduce(self, x):
        return x.norm(dim=-1, keepdim=True)


class ElectronicSpatialExtent(OutputModel, _MassTable):
    """<R^2> = sum_i q_i |r_i - r_com|^2 with per-atom q_i from a two-layer scalar network."""

    def __init__(self, hidden_channels, activation="silu", reduce_op="sum", dtype=torch.float):
        super().__init__(allow_prior_model=False, reduce_op=reduce_op)
        half = hidden_channels // 2
        self.output_network = nn.Sequential(nn.Linear(hidden_channels, half, dtype=dtype),
                                            act_class_mapping[activation](), nn.Linear(half, 1, dtype=dtype))
        self._add_masses(dtype)
        self.reset_parameters()

    def reset_parameters(self):
        for lin in (self.output_network[0], self.output_network[2]):
            nn.init.xavier_uniform_(lin.weight)
            nn.init.zeros_(lin.bias)

    def pre_reduce(self, x, v: Optional[torch.Tensor], z, pos, batch):
        r2 = _offsets_from_centre(self.atomic_mass, z, pos, batch).pow(2).sum(dim=1, keepdim=True)
        return self.output_network(x) * r2


class EquivariantElectronicSpatialExtent(ElectronicSpatialExtent):
    """Same head for equivariant models (the vector features are not used)."""


class EquivariantVectorOutput(EquivariantScalar):
    """One vector per atom: the vector output of the gated blocks."""

    def __init__(self, hidden_channels, activation="silu", reduce_op="sum", dtype=torch.float):
        super().__init__(hidden_channels, activation, allow_prior_model=False, reduce_op="sum", dtype=dtype)

    def pre_reduce(self, x, v, z, pos, batch):
        return self._gated(x, v)[1].squeeze()
