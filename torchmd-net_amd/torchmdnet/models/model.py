"""Model assembly (mirror of reference ``torchmdnet/models/model.py``).

``create_model(args)`` accepts the reference's argument dict (examples/*.yaml keys) and builds the
same module tree in the same order (so seeded initialisation and checkpoints match);
``TorchMD_Net.forward`` returns (y, -dy/dpos) with forces from autograd on ``pos`` exactly as the
reference does (model.py:232-300, ``create_graph=True`` so force losses can be trained).
"""
import re
import warnings
from typing import Dict, List, Optional, Tuple

import torch
from torch import Tensor, nn
from torch.autograd import grad

from . import output_modules
from .utils import dtype_mapping
from .. import priors


def create_model(args, prior_model=None, mean=None, std=None):
    dtype = dtype_mapping[args["precision"]]
    # precision 16 (reference dtype_mapping[16] = float16, models/utils.py:586): parameters and buffers are
    # STORED in float16 (the reference's state_dict dtype), the hot path computes in float32 on upcast copies
    # of them (TorchMD_Net.half_storage_); its outputs are returned in float16
    half = dtype == torch.float16
    if half:
        dtype = torch.float32
    if dtype not in (torch.float32, torch.float64):
        raise NotImplementedError("torchmd-net_amd computes in float32 or float64 (precision 16/32/64)")
    shared_args = dict(
        hidden_channels=args["embedding_dimension"],
        num_layers=args["num_layers"],
        num_rbf=args["num_rbf"],
        rbf_type=args["rbf_type"],
        trainable_rbf=args["trainable_rbf"],
        activation=args["activation"],
        cutoff_lower=args["cutoff_lower"],
        cutoff_upper=args["cutoff_upper"],
        max_z=args["max_z"],
        max_num_neighbors=args["max_num_neighbors"],
        dtype=dtype,
    )
    if args["model"] == "equivariant-transformer":
        from .torchmd_et import TorchMD_ET

        is_equivariant = True
        representation_model = TorchMD_ET(
            attn_activation=args["attn_activation"],
            num_heads=args["num_heads"],
            distance_influence=args["distance_influence"],
            neighbor_embedding=args["neighbor_embedding"],
            **shared_args,
        )
    elif args["model"] == "tensornet":
        from .tensornet import TensorNet

        is_equivariant = False
        representation_model = TensorNet(
            equivariance_invariance_group=args["equivariance_invariance_group"],
            **shared_args,
        )
    elif args["model"] in ("graph-network", "transformer"):
        raise NotImplementedError(f'{args["model"]} is outside the MI355X hot path (ET, TensorNet)')
    else:
        raise ValueError(f'Unknown architecture: {args["model"]}')

    if args.get("atom_filter", -1) > -1:
        raise NotImplementedError("AtomFilter wrapper is outside the hot path")

    if args.get("prior_model") and prior_model is None:
        prior_model = create_prior_models(args)

    output_prefix = "Equivariant" if is_equivariant else ""
    output_model = getattr(output_modules, output_prefix + args["output_model"])(
        args["embedding_dimension"],
        activation=args["activation"],
        reduce_op=args["reduce_op"],
        dtype=dtype,
    )
    model = TorchMD_Net(representation_model, output_model, prior_model=prior_model, mean=mean, std=std,
                        derivative=args["derivative"], dtype=dtype)
    return model.half_storage_() if half else model


def load_model(filepath, args=None, device="cpu", **kwargs):
    """Reference model.py:121-143.  Checkpoints are read with ``weights_only=True``."""
    ckpt = torch.load(filepath, map_location="cpu", weights_only=True)
    if args is None:
        args = ckpt["hyper_parameters"]
    for key, value in kwargs.items():
        if key not in args:
            warnings.warn(f"Unknown hyperparameter: {key}={value}")
        args[key] = value
    model = create_model(args)
    state_dict = {re.sub(r"^model\.", "", k): v for k, v in ckpt["state_dict"].items()}
    if "prior_model.initial_atomref" in state_dict:
        state_dict["prior_model.0.initial_atomref"] = state_dict.pop("prior_model.initial_atomref")
    if "prior_model.atomref.weight" in state_dict:
        state_dict["prior_model.0.atomref.weight"] = state_dict.pop("prior_model.atomref.weight")
    model.load_state_dict(state_dict)
    return model.to(device)


def create_prior_models(args, dataset=None):
    prior_models = []
    if args["prior_model"]:
        prior_model = args["prior_model"]
        prior_names, prior_args = [], []
        if not isinstance(prior_model, list):
            prior_model = [prior_model]
        for prior in prior_model:
            if isinstance(prior, dict):
                for key, value in prior.items():
                    prior_names.append(key)
                    prior_args.append({} if value is None else value)
            else:
                prior_names.append(prior)
                prior_args.append({})
        if "prior_args" in args:
            prior_args = args["prior_args"]
            if not isinstance(prior_args, list):
                prior_args = [prior_args]
        for name, arg in zip(prior_names, prior_args):
            assert hasattr(priors, name), (f"Unknown prior model {name}. "
                                           f"Available models are {', '.join(priors.__all__)}")
            prior_models.append(getattr(priors, name)(dataset=dataset, **arg))
    return prior_models


class TorchMD_Net(nn.Module):
    """Representation model + output head + priors; forces = -d(sum y)/d pos (reference model.py:180-300)."""

    # host-side scratch, not model state: a model that already ran eagerly still scripts
    __jit_ignored_attributes__ = ["_seed_cache"]

    def __init__(self, representation_model, output_model, prior_model=None, mean=None, std=None,
                 derivative=False, dtype=torch.float32):
        super().__init__()
        self.representation_model = representation_model.to(dtype=dtype)
        self.output_model = output_model.to(dtype=dtype)
        if not output_model.allow_prior_model and prior_model is not None:
            prior_model = None
            warnings.warn("Prior model was given but the output model does not allow prior models. "
                          "Dropping the prior model.")
        if isinstance(prior_model, priors.base.BasePrior):
            prior_model = [prior_model]
        self.prior_model = None if prior_model is None else torch.nn.ModuleList(prior_model).to(dtype=dtype)
        self.derivative = derivative
        mean = torch.scalar_tensor(0) if mean is None else mean
        self.register_buffer("mean", mean.to(dtype=dtype))
        std = torch.scalar_tensor(1) if std is None else std
        self.register_buffer("std", std.to(dtype=dtype))
        self.reset_parameters()
        # TorchScript in eval mode: the whole energy + force evaluation as one operator
        # (tmdnet::et_energy_forces) when the configuration is the one it implements
        self.fused_eval = self._fused_eval_capable()
        # precision 16: float16 storage, float32 arithmetic (half_storage_)
        self._half_storage = False
        self._half_inner = False

    @torch.jit.unused
    def half_storage_(self):
        """The reference's precision=16 (``dtype_mapping[16]`` = float16, models/utils.py:586; scripts/train.py:43):
        every floating parameter and buffer is STORED in float16 -- the state_dict a precision-16 reference
        checkpoint holds -- while the HIP kernels (fp32 / fp64 only) compute on float32 upcasts of them, made per
        call (differentiable: gradients reach the float16 parameters through the casts).  Energies and forces
        come back in float16.  Arithmetic is therefore the fp32 path's on fp16-rounded weights; the gate is the
        looser precision-16 one (tests/test_gpu_precision16.py)."""
        self.to(torch.float16)
        self._half_storage = True
        self.fused_eval = False
        return self

    @torch.jit.unused
    def _forward_half(self, z, pos, batch, q, s, extra_args):
        import itertools
        from torch.func import functional_call
        state = {n: (t.float() if t.is_floating_point() else t)
                 for n, t in itertools.chain(self.named_parameters(), self.named_buffers())}
        self._half_inner = True
        try:
            y, neg_dy = functional_call(self, state, (z, pos.float() if pos.is_floating_point() else pos, batch),
                                        {"q": q, "s": s, "extra_args": extra_args}, strict=False)
        finally:
            self._half_inner = False
        return y.half(), (None if neg_dy is None else neg_dy.half())

    @torch.jit.unused
    def _fused_eval_capable(self) -> bool:
        """ET (fp32, fixed RBF basis, the fused stack with a fused out_norm) + EquivariantScalar (the fused head
        kernel's configuration) + plain sum reduction, no priors, forces requested: what tmdnet::et_energy_forces
        evaluates."""
        from .. import kernels
        from .output_modules import EquivariantScalar
        from .torchmd_et import TorchMD_ET
        rep, out = self.representation_model, self.output_model
        if not (self.derivative and self.prior_model is None and type(rep) is TorchMD_ET
                and type(out) is EquivariantScalar):
            return False
        on = rep.out_norm
        return bool(rep.fused_stack and not rep.trainable_rbf and rep.embedding.weight.dtype == torch.float32
                    and len(rep.attention_layers) > 0 and on.elementwise_affine and on.eps == 1e-5
                    and out.reduce_op in ("sum", "add") and kernels.eq_head_fusable(out.output_network)
                    and self.std.numel() == 1 and self.mean.numel() == 1)

    def reset_parameters(self):
        self.representation_model.reset_parameters()
        self.output_model.reset_parameters()
        if self.prior_model is not None:
            for prior in self.prior_model:
                prior.reset_parameters()

    @torch.jit.unused
    def _neg_seed(self, y: Tensor) -> Tensor:
        """The force pass's ``grad_outputs`` (-1 like y, see forward) kept per shape / dtype / device, so
        an energy + force evaluation does not launch a fill for it (read-only: autograd never writes its
        seeds).  Not cached when first needed inside a HIP-graph capture (its memory would belong to
        the graph's pool)."""
        cache = self.__dict__.setdefault("_seed_cache", {})
        key = (tuple(y.shape), y.dtype, y.device)
        t = cache.get(key)
        if t is None:
            t = torch.full_like(y, -1.0)
            if not (y.is_cuda and torch.cuda.is_current_stream_capturing()):
                if len(cache) >= 8:  # bounded: MD / inference over varying molecule counts
                    cache.pop(next(iter(cache)))
                cache[key] = t
        return t

    @torch.jit.unused
    def __getstate__(self):
        # the force-seed cache is device scratch, not model state (torch.save / deepcopy)
        state = self.__dict__.copy()
        state.pop("_seed_cache", None)
        return state

    @torch.jit.unused
    def _early_dim_size(self, batch: Tensor) -> None:
        """The molecule count read back now, while the queue is short: at the reduction the read-back would
        wait out the whole enqueued forward before the force pass could be enqueued (eager evaluation)."""
        if batch.is_cuda and batch.numel() and not torch.cuda.is_current_stream_capturing():
            self.output_model.dim_size_hint = int(batch.max()) + 1

    def forward(self, z: Tensor, pos: Tensor, batch: Optional[Tensor] = None, q: Optional[Tensor] = None,
                s: Optional[Tensor] = None, extra_args: Optional[Dict[str, Tensor]] = None
                ) -> Tuple[Tensor, Optional[Tensor]]:
        assert z.dim() == 1 and z.dtype == torch.long
        batch = torch.zeros_like(z) if batch is None else batch
        if torch.jit.is_scripting():
            if self._half_storage:
                raise RuntimeError("torchmd-net_amd: precision-16 models run eagerly (float16 storage, float32 "
                                   "arithmetic); script a precision-32 copy")
            if self.derivative:
                pos.requires_grad_(True)
            return self._forward_script(z, pos, batch, q, s, extra_args)
        if self._half_storage and not self._half_inner:
            return self._forward_half(z, pos, batch, q, s, extra_args)
        if self.derivative:
            pos.requires_grad_(True)
        self._early_dim_size(batch)
        x, v, z, pos, batch = self.representation_model(z, pos, batch, q=q, s=s)
        fused = None
        if self.prior_model is None:  # the head's tail, x * std, reduce and + mean fused (Scalar)
            fused = self.output_model.fused_head_reduce(x, v, z, pos, batch, self.std, self.mean)
        if fused is None:
            x = self.output_model.pre_reduce(x, v, z, pos, batch)
        if fused is None and self.prior_model is None:  # x * std, reduce and + mean in one pass
            fused = self.output_model.fused_reduce(x, batch, self.std, self.mean)
        if fused is not None:
            x = fused
        else:
            if self.std is not None:
                x = x * self.std
            if self.prior_model is not None:
                for prior in self.prior_model:
                    x = prior.pre_reduce(x, z, pos, batch, extra_args)
            x = self.output_model.reduce(x, batch)
            if self.mean is not None:
                x = x + self.mean
        y = self.output_model.post_reduce(x)
        if self.prior_model is not None:
            for prior in self.prior_model:
                y = prior.post_reduce(y, z, pos, batch, extra_args)
        if self.derivative:
            # -dy/dpos directly: the backward is seeded with -1 instead of negating its result (sign
            # flips are exact; one elementwise launch fewer than the reference's `-dy`, model.py:298)
            grad_outputs: List[Optional[torch.Tensor]] = [self._neg_seed(y)]
            neg_dy = grad([y], [pos], grad_outputs=grad_outputs, create_graph=True, retain_graph=True)[0]
            if neg_dy is None:
                raise RuntimeError("Autograd returned None for the force prediction.")
            return y, neg_dy
        return y, None

    def _forward_script(self, z: Tensor, pos: Tensor, batch: Tensor, q: Optional[Tensor], s: Optional[Tensor],
                        extra_args: Optional[Dict[str, Tensor]]) -> Tuple[Tensor, Optional[Tensor]]:
        """TorchScript body: reference model.py:252-300 line for line (the representation model's
        scripted path runs the HIP operators of libtmdnet_torch.so).  In eval mode a supported ET model runs
        the whole evaluation as ONE operator (tmdnet::et_energy_forces: the eager path's launches issued from
        C++, no autograd graph -- its outputs are not differentiable; script the model in train mode, or set
        ``fused_eval = False`` before scripting, to differentiate the forces)."""
        if self.fused_eval and not self.training and pos.is_cuda and pos.dtype == torch.float32:
            return self.representation_model.fused_energy_forces(z, pos, batch, self.output_model.head_params(),
                                                                 self.std, self.mean)
        x, v, z, pos, batch = self.representation_model(z, pos, batch, q=q, s=s)
        x = self.output_model.pre_reduce(x, v, z, pos, batch)
        if self.std is not None:
            x = x * self.std
        prior_model = self.prior_model
        if prior_model is not None:
            for prior in prior_model:
                x = prior.pre_reduce(x, z, pos, batch, extra_args)
        x = self.output_model.reduce(x, batch)
        if self.mean is not None:
            x = x + self.mean
        y = self.output_model.post_reduce(x)
        if prior_model is not None:
            for prior in prior_model:
                y = prior.post_reduce(y, z, pos, batch, extra_args)
        if self.derivative:
            grad_outputs: List[Optional[torch.Tensor]] = [torch.ones_like(y)]
            dy = grad([y], [pos], grad_outputs=grad_outputs, create_graph=True, retain_graph=True)[0]
            if dy is None:
                raise RuntimeError("Autograd returned None for the force prediction.")
            return y, -dy
        return y, None
