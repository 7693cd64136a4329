"""Data-parallel training step (replaces the reference's Lightning LNNP + DDPStrategy for the hot path).

Reference: LNNP.step (torchmdnet/module.py:130-179: energy / force MSE, weighted), optimizer_step
linear LR warm-up (module.py:181-193), AdamW (module.py:40-59), DDP over NCCL
(scripts/train.py:175-189; DDP broadcasts rank 0's parameters and buffers when it wraps the model).

MI355X design: one process per GPU (torchrun or ``bench.py --gpus N``), RCCL ("nccl" backend) over
xGMI.  The gradients of ET-QM9-128 are 7.5 MB, ET-SPICE 4.9 MB: ONE flat all-reduce per step (a
single ring pass bounded by one 153 GB/s xGMI link is ~50 us) instead of DDP's bucket hooks, which
at this size only add launches.  Every parameter's ``.grad`` IS a view of that flat buffer, so
autograd accumulates straight into it and the all-reduce needs no copies in or out.  AdamW is the
fused multi-tensor kernel; its ``found_inf`` input skips a step on the device (no host sync) when a
static-capacity neighbour list overflowed on any rank.
"""
import torch
import torch.distributed as dist
import torch.nn.functional as F

from . import _native, kernels
from . import et_stack
from .et_stack import second_order_expected


def _world(group=None):
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group)
    return 1


def broadcast_parameters(module, src=0, group=None):
    """Copy rank ``src``'s parameters and floating buffers to every rank (what DDP does when it wraps
    the model, so replicas start identical whatever their seeds).  One flat broadcast."""
    if _world(group) == 1:
        return
    ts = [t for t in list(module.parameters()) + list(module.buffers()) if t.is_floating_point()]
    if not ts:
        return
    with torch.no_grad():
        by_dtype = {}
        for t in ts:
            by_dtype.setdefault(t.dtype, []).append(t)
        for dtype in sorted(by_dtype, key=str):
            group_ts = by_dtype[dtype]
            flat = torch.cat([t.detach().reshape(-1) for t in group_ts])
            dist.broadcast(flat, src, group=group)
            off = 0
            for t in group_ts:
                n = t.numel()
                t.copy_(flat[off:off + n].view_as(t))
                off += n


class GradAllReduce:
    """Fused average of all parameter gradients across the process group (one RCCL call).

    ``flat`` holds every gradient plus one trailing slot, the step-skip flag (> 0 after the sum when
    any rank flagged its step).  ``p.grad`` of every parameter is bound to its view of ``flat``:
    backward accumulates in place, ``__call__`` all-reduces the buffer itself.  A ``.grad`` that is
    not the view (set to None by ``zero_grad``, or replaced by a caller) is copied in and rebound."""

    def __init__(self, params, group=None):
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        n = sum(p.numel() for p in self.params)
        dev = self.params[0].device
        self.flat = torch.zeros(n + 1, dtype=self.params[0].dtype, device=dev)
        self.views = []
        off = 0
        for p in self.params:
            self.views.append(self.flat[off:off + p.numel()].view_as(p))
            off += p.numel()
        self.flag = self.flat[n:]
        self.bind()

    def bind(self):
        """Make every ``p.grad`` the flat buffer's view (keeping the current gradient values)."""
        with torch.no_grad():
            for p, v in zip(self.params, self.views):
                g = p.grad
                if g is None:
                    v.zero_()
                elif g.data_ptr() != v.data_ptr():
                    v.copy_(g)
                p.grad = v

    def __call__(self):
        if _world(self.group) == 1:
            return
        self.bind()
        dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=self.group)
        self.flat.div_(_world(self.group))

    # --- two buckets, the optimizer overlapped with the second all-reduce (world > 1)
    def split_params(self, frac=0.5):
        """(tail, head) parameter lists of a two-bucket split: the TAIL bucket is the flat buffer's end
        (the last parameters and the skip flag) and is reduced first, so the optimizer over its
        parameters -- which needs the reduced flag -- can run while the HEAD bucket is reduced."""
        n = sum(p.numel() for p in self.params)
        cut, off, k = int(n * frac), 0, 0
        for i, p in enumerate(self.params):
            if off >= cut:
                k = i
                break
            off += p.numel()
        else:
            k = len(self.params)
        self._cut = off  # flat[:off] = head bucket, flat[off:] = tail bucket (incl. the flag)
        return self.params[k:], self.params[:k]

    def reduce_overlapped(self, first, second):
        """All-reduce the tail bucket, then the head bucket, on a side stream (RCCL over xGMI); ``first()``
        (the optimizer step of the tail's parameters) runs on the current stream as soon as the tail is
        averaged, overlapped with the head's all-reduce, then ``second()``.  World 1: both steps, no
        collective.  CPU (gloo): the same order without streams."""
        ws = _world(self.group)
        if ws == 1:
            first()
            second()
            return
        self.bind()
        tail, head = self.flat[self._cut:], self.flat[:self._cut]
        if not self.flat.is_cuda:
            dist.all_reduce(tail, op=dist.ReduceOp.SUM, group=self.group)
            tail.div_(ws)
            first()
            if head.numel():
                dist.all_reduce(head, op=dist.ReduceOp.SUM, group=self.group)
                head.div_(ws)
            second()
            return
        cur = torch.cuda.current_stream(self.flat.device)
        side = getattr(self, "_side", None)
        if side is None:
            side = self._side = torch.cuda.Stream(device=self.flat.device)
        side.wait_stream(cur)  # the gradients are complete
        with torch.cuda.stream(side):
            dist.all_reduce(tail, op=dist.ReduceOp.SUM, group=self.group)
            ev_tail = torch.cuda.Event()
            ev_tail.record(side)
            if head.numel():
                dist.all_reduce(head, op=dist.ReduceOp.SUM, group=self.group)
            ev_head = torch.cuda.Event()
            ev_head.record(side)
        cur.wait_event(ev_tail)
        tail.div_(ws)
        first()
        cur.wait_event(ev_head)
        head.div_(ws)
        second()
        # the buffer is rewritten by the next backward on `cur`: the side stream's use of it must end first
        tail.record_stream(side)
        head.record_stream(side)


class SplitAdamW(torch.optim.Optimizer):
    """Two fused AdamW instances over the tail / head buckets of ``GradAllReduce.split_params`` (the
    same per-parameter update as one AdamW: it is elementwise), so the tail's update can overlap the
    head bucket's all-reduce.  A torch Optimizer (schedulers such as ReduceLROnPlateau accept it) whose
    param_groups ARE the parts' groups (an LR change reaches them)."""

    def __init__(self, tail, head, lr, weight_decay):
        # fixed roles: parts[0] = TAIL (stepped by step_part(0) once the tail bucket is averaged), parts[1] =
        # HEAD; an empty bucket keeps its slot as None -- dropping it would shift the head optimizer into
        # slot 0 and step it before the head bucket's all-reduce finished (un-averaged gradients)
        parts = [_adamw(ps, lr, weight_decay) if ps else None for ps in (tail, head)]
        live = [o for o in parts if o is not None]
        super().__init__([g for o in live for g in o.param_groups], dict(lr=lr, weight_decay=weight_decay))
        self.parts = parts
        self.param_groups = [g for o in live for g in o.param_groups]  # the same dict objects

    def __setattr__(self, k, v):
        if k in ("found_inf", "grad_scale"):
            for o in self.__dict__.get("parts", []):
                if o is not None:
                    setattr(o, k, v)
        super().__setattr__(k, v)

    def zero_grad(self, set_to_none=True):
        for o in self.parts:
            if o is not None:
                o.zero_grad(set_to_none=set_to_none)

    def step(self, closure=None):
        for o in self.parts:
            if o is not None:
                o.step()

    def step_part(self, i):
        if self.parts[i] is not None:
            self.parts[i].step()

    def state_dict(self):
        return {"parts": [None if o is None else o.state_dict() for o in self.parts]}

    def load_state_dict(self, sd):
        for o, d in zip(self.parts, sd["parts"]):
            if o is not None and d is not None:
                o.load_state_dict(d)


def _make_optimizer(reduce, lr, weight_decay):
    """One fused AdamW at world 1; at world > 1 the two-bucket SplitAdamW whose tail update overlaps
    the head bucket's all-reduce (``step_reduce``)."""
    if _world(reduce.group) > 1:
        tail, head = reduce.split_params()
        return SplitAdamW(tail, head, lr, weight_decay)
    return _adamw(reduce.params, lr, weight_decay)


def step_reduce(reduce, opt, before_first=None):
    """All-reduce the gradients and step the optimizer: with a SplitAdamW the tail bucket's update runs
    while the head bucket is still being reduced (world > 1); ``before_first()`` runs once the tail
    (which holds the skip flag) is averaged."""
    if isinstance(opt, SplitAdamW):
        def first():
            if before_first is not None:
                before_first()
            opt.step_part(0)
        reduce.reduce_overlapped(first, lambda: opt.step_part(1))
    else:
        reduce()
        if before_first is not None:
            before_first()
        opt.step()
    # fused AdamW writes the parameters without bumping their version counters: the C++ et_stack
    # operator's packed weights (TorchScript / eval-mode eager) must not outlive this step
    _native.invalidate_stack_cache()


def _adamw(params, lr, weight_decay):
    dev = params[0].device
    # the fused multi-tensor AdamW (one launch per dtype group; honours found_inf on the device)
    return torch.optim.AdamW(params, lr=lr, weight_decay=weight_decay, fused=dev.type == "cuda")


def _copy_grads(pairs):
    """Copy (flat-buffer view, gradient) pairs: ONE multi-tensor launch for the contiguous gradients (a
    single strided one, e.g. a column block of a weight-gradient GEMM's output, would send the whole
    list down the per-tensor path: one copy launch each), the strided ones one by one."""
    fast = [(v, g) for v, g in pairs if g.is_contiguous()]
    if fast:
        torch._foreach_copy_([v for v, _ in fast], [g for _, g in fast])
    for v, g in pairs:
        if not g.is_contiguous():
            v.copy_(g)


class LNNPStep:
    """One optimisation step of the reference training objective on a batch of molecules."""

    def __init__(self, model, lr=4e-4, weight_decay=0.0, y_weight=1.0, neg_dy_weight=1.0,
                 lr_warmup_steps=0, group=None):
        self.model = model
        self.y_weight = y_weight
        self.neg_dy_weight = neg_dy_weight
        self.lr = lr
        self.lr_warmup_steps = lr_warmup_steps
        broadcast_parameters(model, 0, group)
        self.reduce = GradAllReduce(model.parameters(), group)
        self.opt = _make_optimizer(self.reduce, lr, weight_decay)
        self.global_step = 0

    def loss(self, z, pos, batch, y, neg_dy):
        # a force loss differentiates the force pass again: let the ET stack record for its hand second order
        with second_order_expected(self.neg_dy_weight > 0):
            pred, pred_neg_dy = self.model(z, pos, batch)
        if y.ndim == 1:  # reference module.py:147-148
            y = y.unsqueeze(1)
        if (self.y_weight > 0 and self.neg_dy_weight > 0 and pred_neg_dy is not None and pred.is_cuda
                and pred.shape == y.shape and pred_neg_dy.shape == neg_dy.shape
                and all(t.dtype == pred.dtype and t.device == pred.device for t in (y, pred_neg_dy, neg_dy))):
            # both terms in one launch (and one for their backward): kernels.mse2
            return kernels.mse2(pred, y, pred_neg_dy, neg_dy, self.y_weight, self.neg_dy_weight)
        loss = 0.0
        if self.y_weight > 0:
            loss = loss + self.y_weight * F.mse_loss(pred, y)
        if self.neg_dy_weight > 0 and pred_neg_dy is not None:
            loss = loss + self.neg_dy_weight * F.mse_loss(pred_neg_dy, neg_dy)
        return loss

    def backward(self, loss):
        # gradients of the parameters only: the positions are a leaf too (forces need them), but
        # accumulating a position gradient nobody reads is wasted work -- and under HIP-graph
        # capture the positions' AccumulateGrad would run across streams
        loss.backward(inputs=self.reduce.params)
        et_stack.check_pending_consumed()

    def _warmup_lr(self):
        if self.lr_warmup_steps and self.global_step < self.lr_warmup_steps:
            scale = min(1.0, float(self.global_step + 1) / float(self.lr_warmup_steps))
            for g in self.opt.param_groups:
                g["lr"] = scale * self.lr

    def step(self, z, pos, batch, y, neg_dy):
        self.opt.zero_grad(set_to_none=False)  # zeroes the flat buffer's views in place
        loss = self.loss(z, pos, batch, y, neg_dy)
        self.backward(loss)
        self._warmup_lr()
        step_reduce(self.reduce, self.opt)
        self.global_step += 1
        return loss.detach()


class GraphedTrainStep(LNNPStep):
    """LNNPStep with the forward, the force pass and the whole (double) backward captured in ONE
    HIP graph for a fixed batch layout (same z / batch / label shapes every step, e.g. a padded or
    fixed-size loader).  Per step: copy the inputs in, replay, then the fused RCCL all-reduce and
    the fused AdamW run eagerly (the collective stays outside the graph).  The neighbour list runs in
    its static-capacity mode (capacity = margin x the warm-up pair count); the molecule count of
    ``reduce`` is frozen from warm-up as in inference capture (reference output_modules.py:27-43).
    The graph writes the parameter gradients straight into the all-reduce buffer (one multi-tensor
    copy) and raises the buffer's skip flag when the pair count exceeded the capacity; the flag is
    summed over ranks with the gradients and AdamW skips the step on the device when it is set
    (weights untouched; ``skipped_steps`` counts them, ``check_capacity`` raises).

    Drop every reference to an earlier loss / autograd graph of this model before constructing it:
    a live graph keeps the parameters' AccumulateGrad nodes (bound to the stream they were created
    on) alive, and a capture that reaches them across streams is invalid."""

    def __init__(self, model, z, pos, batch, y, neg_dy, margin=1.25, warmup=3, **kw):
        import math
        super().__init__(model, **kw)
        from .graphs import _distance_modules
        self.z, self.batch = z.clone(), batch.clone()
        self.pos = pos.detach().clone()
        self.y = y.detach().clone()
        self.neg_dy = neg_dy.detach().clone()
        dev = pos.device
        rep = model.representation_model
        # eager warm-up on a CLONE of the positions (sizes the edge capacity, freezes the molecule
        # count of reduce): the captured positions' AccumulateGrad must not be created on the
        # default stream before the capture
        self.opt.zero_grad(set_to_none=True)
        self.backward(self.loss(self.z, self.pos.clone(), self.batch, self.y, self.neg_dy))
        g = rep.distance.graph(self.pos.clone(), self.batch)
        self.edge_capacity = int(math.ceil(g.num_pairs * margin / 256.0) * 256)
        del g
        self.dists = _distance_modules(model)
        for d in self.dists:
            d.static_capacity = self.edge_capacity
        try:
            torch.autograd.graph.set_warn_on_accumulate_grad_stream_mismatch(False)
        except AttributeError:
            pass
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self.opt.zero_grad(set_to_none=True)
                self.backward(self.loss(self.z, self.pos, self.batch, self.y, self.neg_dy))
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize(dev)
        # the parameter gradients are graph OUTPUTS (autograd.grad, as make_graphed_callables does):
        # no AccumulateGrad node runs inside the capture; the graph copies them into the flat buffer
        self.opt.zero_grad(set_to_none=True)
        params = self.reduce.params
        self.reduce.flat.zero_()
        # the backward's seed: allocated outside the graph and kept alive with it (its replays read it)
        self._seed = seed = torch.ones((), dtype=params[0].dtype, device=dev)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, capture_error_mode="thread_local"):
            self.static_loss = self.loss(self.z, self.pos, self.batch, self.y, self.neg_dy)
            grads = torch.autograd.grad(self.static_loss, params, grad_outputs=seed.expand_as(self.static_loss),
                                        allow_unused=True)
            pairs = [(v, g) for v, g in zip(self.reduce.views, grads) if g is not None]
            _copy_grads(pairs)
            ov = rep.distance.last_overflow
            self.reduce.flag.copy_(ov.num.reshape(1) > ov.capacity)
        torch.cuda.synchronize(dev)
        del grads, pairs
        self.reduce.bind()
        self.overflow = rep.distance.last_overflow
        self.found_inf = torch.zeros((), dtype=torch.float32, device=dev)
        self.skip_count = torch.zeros((), dtype=torch.float32, device=dev)
        self.opt.found_inf = self.found_inf
        self.opt.grad_scale = None

    def step(self, z=None, pos=None, batch=None, y=None, neg_dy=None):
        with torch.no_grad():
            for name, dst, src in (("z", self.z, z), ("pos", self.pos, pos), ("batch", self.batch, batch),
                                   ("y", self.y, y), ("neg_dy", self.neg_dy, neg_dy)):
                if src is None:
                    continue
                if name == "y" and src.ndim == 1:
                    src = src.unsqueeze(1)
                if src.shape != dst.shape:
                    raise ValueError(f"GraphedTrainStep: {name} has shape {tuple(src.shape)}, the captured "
                                     f"layout is {tuple(dst.shape)}")
                dst.copy_(src)
        self.graph.replay()
        self._warmup_lr()

        def flag():  # skip flag (> 0 on any rank) -> AdamW's found_inf (exactly 1.0 or 0.0)
            self.found_inf.copy_(self.reduce.flag[0].sign())
            self.skip_count.add_(self.found_inf)

        step_reduce(self.reduce, self.opt, flag)
        self.global_step += 1
        return self.static_loss.detach()

    @property
    def skipped_steps(self):
        return int(self.skip_count.item())

    def check_capacity(self):
        """Raises (host sync) if a replay's neighbour list exceeded the captured capacity: the
        latest step, or any earlier one (whose AdamW update was skipped)."""
        if bool(self.overflow.item()) or self.skipped_steps:
            raise RuntimeError(f"neighbour pairs exceed the captured edge capacity {self.edge_capacity} "
                               f"({self.skipped_steps} optimizer steps skipped)")

    def release(self):
        for d in self.dists:
            d.static_capacity = None


# ----------------------------------------------------------------------------- variable-size batches, captured
class PaddedBatches:
    """Fixed-shape layouts of variable-size molecule batches, so a training step can be ONE graph replay
    (VERDICT r3 "next" #4).

    Reference batches are PyG collations of whatever molecules the sampler draws (data.py:138-144): the
    atom count changes every step, and a captured step needs fixed shapes.  A batch is padded to the
    smallest capacity of ``atom_buckets`` that holds it (one captured graph per capacity used) with GHOST
    atoms: all on one dummy molecule (index ``max_molecules``), hydrogen, placed on a line far from
    everything and ``2 * cutoff`` apart -- every ghost sees only its own self loop, so no real atom's
    energy or force changes.  The molecule axis is padded to ``max_molecules + 1`` rows (empty molecules
    reduce to 0).  ``wy`` / ``wf`` weight the squared errors so that the weighted sums are the reference's
    MEAN losses over the real entries only (module.py:174-177): ``wy = 1 / n_mol`` on real molecules,
    ``wf = 1 / (3 n_atoms)`` on real atoms, 0 on padding.  ``collate`` is a DataLoader collate_fn (it
    runs in the loader's workers)."""

    GHOST_ORIGIN = 1.0e4  # far from any molecule (Angstrom)

    def __init__(self, atom_buckets, max_molecules, cutoff):
        self.buckets = sorted(int(a) for a in atom_buckets)
        self.max_molecules = int(max_molecules)
        self.spacing = 2.0 * float(cutoff) + 1.0

    def capacity(self, n_atoms):
        for a in self.buckets:
            if a >= n_atoms + 1:  # at least one ghost: the dummy molecule is never empty
                return a
        raise ValueError(f"batch of {n_atoms} atoms exceeds the largest atom bucket {self.buckets[-1]}")

    def collate(self, samples):
        from .data import Data
        n_mol = len(samples)
        if n_mol > self.max_molecules:
            raise ValueError(f"{n_mol} molecules > max_molecules {self.max_molecules}")
        n_at = sum(int(s.z.shape[0]) for s in samples)
        A, M = self.capacity(n_at), self.max_molecules
        ng = A - n_at
        dtype = samples[0].pos.dtype
        z = torch.ones(A, dtype=torch.long)
        z[:n_at] = torch.cat([s.z.reshape(-1).long() for s in samples])
        pos = torch.zeros(A, 3, dtype=dtype)
        pos[:n_at] = torch.cat([s.pos.reshape(-1, 3) for s in samples])
        pos[n_at:, 0] = self.GHOST_ORIGIN + self.spacing * torch.arange(ng, dtype=dtype)
        pos[n_at:, 1:] = self.GHOST_ORIGIN
        batch = torch.full((A,), M, dtype=torch.long)
        batch[:n_at] = torch.cat([torch.full((int(s.z.shape[0]),), i, dtype=torch.long)
                                  for i, s in enumerate(samples)])
        out = Data(z=z, pos=pos, batch=batch, n_atoms=n_at, n_mol=n_mol, capacity=A)
        wy = torch.zeros(M + 1, 1, dtype=dtype)
        wy[:n_mol] = 1.0 / n_mol
        wf = torch.zeros(A, 1, dtype=dtype)
        wf[:n_at] = 1.0 / (3 * n_at)
        out.wy, out.wf = wy, wf
        if "y" in samples[0]:
            y = torch.zeros(M + 1, 1, dtype=dtype)
            y[:n_mol] = torch.cat([s.y.reshape(1, -1) for s in samples]).to(dtype)
            out.y = y
        if "neg_dy" in samples[0]:
            f = torch.zeros(A, 3, dtype=dtype)
            f[:n_at] = torch.cat([s.neg_dy.reshape(-1, 3) for s in samples]).to(dtype)
            out.neg_dy = f
        return out


def padded_losses(pred, neg_dy, b):
    """(L_y, L_f): the reference's mean-squared energy / force losses of a padded batch (weights 0 on
    the padding, so the sums are means over the real entries)."""
    ly = (b.wy * (pred - b.y) ** 2).sum() if "y" in b else pred.sum() * 0
    # an energy-only model (derivative=False) returns no forces: the force term is a zero scalar
    lf = (b.wf * (neg_dy - b.neg_dy) ** 2).sum() if ("neg_dy" in b and neg_dy is not None) else pred.sum() * 0
    return ly, lf


def pad_shift(model, n_atoms, capacity):
    """Host value of TensorNet's padded-batch pair-count correction (``TensorNet._pad_shift``).

    The reference's static_shapes mode sends every unused slot of the ``max_num_pairs(N)`` capacity to
    atom 0 as a (0, 0) edge (tensornet.py:215-221).  For the real molecules alone that is
    ``max_pairs(n_real) - pairs_real`` slots; a padded batch of ``capacity`` atoms has
    ``max_pairs(capacity) - (pairs_real + n_ghosts)`` (each ghost has its self loop).  Adding
    ``max_pairs(capacity) - max_pairs(n_real) - n_ghosts`` to the pair count restores the real count."""
    d = model.representation_model.distance
    return d._max_pairs(int(capacity)) - d._max_pairs(int(n_atoms)) - (int(capacity) - int(n_atoms))


class _BucketStep:
    """One captured training step for one atom capacity: static inputs, graph, raw loss outputs."""

    def __init__(self, model, params, views, flag, b, scale_y, scale_f, margin, warmup, min_capacity=0):
        import math
        from .graphs import _distance_modules
        dev = params[0].device
        self.inputs = {k: getattr(b, k).to(dev).clone() for k in ("z", "pos", "batch", "wy", "wf", "y", "neg_dy")
                       if k in b}
        rep = model.representation_model
        self.model = model
        # TensorNet static_shapes: its atom-0 padding multiplicity must count the real atoms only
        self.pad_shift = None
        if getattr(rep, "static_shapes", False) and hasattr(rep, "_pad_shift"):
            self.pad_shift = torch.zeros(1, dtype=torch.int32, device=dev)
            self._set_shift(b)
        dists = _distance_modules(model)
        bs = _Static(self.inputs)

        def loss_fn():
            with second_order_expected(scale_f > 0):
                pred, nd = model(bs.z, bs.pos, bs.batch)
            ly, lf = padded_losses(pred, nd, bs)
            return ly, lf, ly * scale_y + lf * scale_f

        # (try / finally: a warm-up or capture that raises must not leave the static capacity or TensorNet's
        # padded-batch shift set for later eager calls, e.g. validation on unpadded batches)
        grads = pairs = None
        try:
            # eager warm-up on a clone of the positions (sizes the edge capacity, freezes the molecule count
            # of reduce): the captured positions' autograd state must not start on the default stream
            for d in dists:
                d.static_capacity = None
            g = rep.distance.graph(bs.pos.clone(), bs.batch)
            self.edge_capacity = max(int(math.ceil(g.num_pairs * margin / 256.0) * 256), int(min_capacity))
            del g
            pos0 = bs.pos
            bs.pos = pos0.clone()
            torch.autograd.grad(loss_fn()[2], params, allow_unused=True)
            bs.pos = pos0
            for d in dists:
                d.static_capacity = self.edge_capacity
            s = torch.cuda.Stream(device=dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                for _ in range(warmup):
                    torch.autograd.grad(loss_fn()[2], params, allow_unused=True)
            torch.cuda.current_stream(dev).wait_stream(s)
            torch.cuda.synchronize(dev)
            # the backward's seed: allocated outside the graph and kept alive with it (its replays read it)
            self._seed = seed = torch.ones((), dtype=params[0].dtype, device=dev)
            self.graph = torch.cuda.CUDAGraph()
            # thread-local capture: the data loader's pin-memory thread keeps issuing host-allocation and copy calls
            # while a new bucket is captured mid-epoch (global mode invalidated such a capture under a profiler)
            with torch.cuda.graph(self.graph, capture_error_mode="thread_local"):
                self.ly, self.lf, total = loss_fn()
                grads = torch.autograd.grad(total, params, grad_outputs=seed.expand_as(total), allow_unused=True)
                pairs = [(v, gr) for v, gr in zip(views, grads) if gr is not None]
                zero = [v for v, gr in zip(views, grads) if gr is None]
                _copy_grads(pairs)
                if zero:
                    torch._foreach_zero_(zero)
                ov = rep.distance.last_overflow
                flag.copy_(ov.num.reshape(1) > ov.capacity)
            torch.cuda.synchronize(dev)
        finally:
            for d in dists:
                d.static_capacity = None
            if self.pad_shift is not None:
                rep._pad_shift = None  # the graph keeps reading self.pad_shift; eager calls see no shift
        del grads, pairs

    def _set_shift(self, b):
        v = pad_shift(self.model, b.n_atoms, b.capacity)
        self.pad_shift.fill_(v)
        self.model.representation_model._pad_shift = (self.pad_shift, v)

    def load(self, b):
        with torch.no_grad():
            for k, dst in self.inputs.items():
                dst.copy_(getattr(b, k), non_blocking=True)
            if self.pad_shift is not None:
                self.pad_shift.fill_(pad_shift(self.model, b.n_atoms, b.capacity))


class _Static:
    def __init__(self, d):
        self.__dict__.update(d)

    def __contains__(self, k):
        return k in self.__dict__


class PaddedGraphedTrainer:
    """Training steps of variable-size molecule batches as graph replays (the reference LNNP.step +
    DDP all-reduce + AdamW, module.py:130-193): batches from ``PaddedBatches.collate``, one captured
    step per atom capacity (captured on first use), the RCCL all-reduce and the fused AdamW eager.

    Overflow of the static neighbour-list capacity is exact, not lossy: the captured step raises the
    all-reduce buffer's flag, AdamW skips on the device (on every rank: the flag is summed), and before
    the NEXT step the host reads the flag (by then the step has long finished: the host collated the
    next batch meanwhile), recaptures the overflowing capacity 1.5x larger and re-runs the same batch --
    every batch is applied once, in order, as in the eager loop."""

    def __init__(self, model, batches, lr=4e-4, weight_decay=0.0, y_weight=1.0, neg_dy_weight=1.0,
                 ema_alpha_y=1.0, ema_alpha_neg_dy=1.0, lr_warmup_steps=0, margin=1.3, warmup=2, group=None):
        self.model, self.batches = model, batches
        self.y_weight, self.neg_dy_weight = float(y_weight), float(neg_dy_weight)
        self.alpha_y, self.alpha_f = float(ema_alpha_y), float(ema_alpha_neg_dy)
        self.lr, self.lr_warmup_steps = lr, lr_warmup_steps
        self.margin, self.warmup = margin, warmup
        broadcast_parameters(model, 0, group)
        self.reduce = GradAllReduce(model.parameters(), group)
        self.opt = _make_optimizer(self.reduce, lr, weight_decay)
        dev = self.reduce.flat.device
        self.found_inf = torch.zeros((), dtype=torch.float32, device=dev)
        self.opt.found_inf = self.found_inf
        self.opt.grad_scale = None
        self.steps = {}
        self.ema = {}
        self.global_step = 0
        self.recaptures = 0
        self._pending = None  # (batch, flag copy, event) of the last step, checked before the next
        self._flag_host = torch.zeros(1, dtype=self.reduce.flat.dtype).pin_memory() if torch.cuda.is_available() \
            else torch.zeros(1, dtype=self.reduce.flat.dtype)
        try:
            torch.autograd.graph.set_warn_on_accumulate_grad_stream_mismatch(False)
        except AttributeError:
            pass

    def _capture(self, b, min_capacity=0):
        # the EMA of the reference scales each loss term's gradient by alpha (module.py:112-128)
        sy = self.y_weight * self.alpha_y if self.y_weight > 0 else 0.0
        sf = self.neg_dy_weight * self.alpha_f if self.neg_dy_weight > 0 else 0.0
        self.reduce.bind()
        st = _BucketStep(self.model, self.reduce.params, self.reduce.views, self.reduce.flag, b, sy, sf, self.margin,
                         self.warmup, min_capacity)
        self.reduce.bind()
        self.steps[int(b.capacity)] = st
        return st

    def _run(self, b, gs):
        """Replay (capturing first if needed) the step of batch ``b`` as global step ``gs`` (the warm-up
        schedule's index), all-reduce, AdamW (skipped on the device on overflow)."""
        st = self.steps.get(int(b.capacity))
        if st is None:
            st = self._capture(b)
        st.load(b)
        st.graph.replay()
        if self.lr_warmup_steps and gs < self.lr_warmup_steps:
            scale = min(1.0, float(gs + 1) / float(self.lr_warmup_steps))
            for g in self.opt.param_groups:
                g["lr"] = scale * self.lr
        step_reduce(self.reduce, self.opt, lambda: self.found_inf.copy_(self.reduce.flag[0].sign()))
        self._flag_host.copy_(self.reduce.flag, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return st, ev

    def _loss_terms(self, st):
        """(L_y, L_f, total) of the replayed step with the reference's EMA (updates ``self.ema``)."""
        ly, lf = st.ly.detach().clone(), st.lf.detach().clone()
        out = []
        for kind, raw, alpha in (("y", ly, self.alpha_y), ("neg_dy", lf, self.alpha_f)):
            if alpha < 1:
                prev = self.ema.get(kind, raw)
                raw = alpha * raw + (1 - alpha) * prev
                self.ema[kind] = raw.detach()
            out.append(raw)
        return [out[0], out[1], out[0] * self.y_weight + out[1] * self.neg_dy_weight]

    def _settle(self):
        """Check the previous step's overflow flag; recapture + redo it if it was skipped.  The redo runs
        as the same global step from the same EMA state and writes its losses INTO the device scalars the
        skipped step returned."""
        while self._pending is not None:
            b, ev, gs, ema0, outs = self._pending
            ev.synchronize()
            if float(self._flag_host[0]) <= 0:
                self._pending = None
                return
            # skipped on every rank: a bigger capacity for this layout, the same batch again
            old = self.steps.pop(int(b.capacity))
            need = int(old.edge_capacity * 1.5)
            del old
            self.recaptures += 1
            self._capture(b, need)
            self.ema = dict(ema0)
            st, ev = self._run(b, gs)
            for o, n in zip(outs, self._loss_terms(st)):
                o.copy_(n)
            self._pending = (b, ev, gs, ema0, outs)

    def step(self, b):
        """One training step on a padded device batch; returns (L_y, L_f, total) device scalars (the
        reported loss applies the reference's EMA).  They are final once the NEXT ``step`` (or
        ``finish``) has returned: a step found to have overflowed the edge capacity is redone then, and
        its losses are rewritten in place."""
        self._settle()
        gs = self.global_step
        ema0 = dict(self.ema)
        st, ev = self._run(b, gs)
        outs = self._loss_terms(st)
        self._pending = (b, ev, gs, ema0, outs)
        self.global_step += 1
        return tuple(outs)

    def finish(self):
        self._settle()
