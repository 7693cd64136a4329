"""Data-parallel training step (replaces the reference's Lightning LNNP + DDPStrategy for the hot path).

Reference: LNNP.step (torchmdnet/module.py:130-179: energy / force MSE, weighted), optimizer_step
linear LR warm-up (module.py:181-193), AdamW (module.py:40-59), DDP over NCCL
(scripts/train.py:175-189).

MI355X design: one process per GPU (torchrun), RCCL ("nccl" backend) over xGMI.  The gradients of
ET-QM9-128 are 7.5 MB, ET-SPICE 4.9 MB: ONE flat all-reduce per step (a single ring pass bounded by
one 153 GB/s xGMI link is ~50 us) instead of DDP's bucket hooks, which at this size only add launch
overhead.  Gradients are flattened into a persistent buffer (no per-step allocation).
"""
import torch
import torch.distributed as dist
import torch.nn.functional as F


class GradAllReduce:
    """Fused average of all parameter gradients across the process group (one RCCL call)."""

    def __init__(self, params, group=None):
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        n = sum(p.numel() for p in self.params)
        dev = self.params[0].device
        self.flat = torch.zeros(n, dtype=self.params[0].dtype, device=dev)

    def __call__(self):
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(self.group) == 1:
            return
        off = 0
        views = []
        for p in self.params:
            n = p.numel()
            v = self.flat[off:off + n]
            if p.grad is None:
                v.zero_()
            else:
                v.copy_(p.grad.reshape(-1))
            views.append(v)
            off += n
        dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=self.group)
        self.flat.div_(dist.get_world_size(self.group))
        for p, v in zip(self.params, views):
            if p.grad is None:
                p.grad = v.view_as(p).clone()
            else:
                p.grad.copy_(v.view_as(p))


class LNNPStep:
    """One optimisation step of the reference training objective on a batch of molecules."""

    def __init__(self, model, lr=4e-4, weight_decay=0.0, y_weight=1.0, neg_dy_weight=1.0,
                 lr_warmup_steps=0, group=None):
        self.model = model
        self.y_weight = y_weight
        self.neg_dy_weight = neg_dy_weight
        self.lr = lr
        self.lr_warmup_steps = lr_warmup_steps
        self.opt = torch.optim.AdamW(model.parameters(), lr=lr, weight_decay=weight_decay)
        self.reduce = GradAllReduce(model.parameters(), group)
        self.global_step = 0

    def loss(self, z, pos, batch, y, neg_dy):
        pred, pred_neg_dy = self.model(z, pos, batch)
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

    def step(self, z, pos, batch, y, neg_dy):
        self.opt.zero_grad(set_to_none=False)
        loss = self.loss(z, pos, batch, y, neg_dy)
        self.backward(loss)
        self.reduce()
        if self.lr_warmup_steps and self.global_step < self.lr_warmup_steps:
            scale = min(1.0, float(self.global_step + 1) / float(self.lr_warmup_steps))
            for g in self.opt.param_groups:
                g["lr"] = scale * self.lr
        self.opt.step()
        self.global_step += 1
        return loss.detach()


class GraphedTrainStep(LNNPStep):
    """LNNPStep with the forward, the force pass and the whole (double) backward captured in ONE
    HIP graph for a fixed batch layout (same z / batch / label shapes every step, e.g. a padded or
    fixed-size loader).  Per step: copy the inputs in, replay, then the fused RCCL all-reduce and
    AdamW run eagerly (the collective stays outside the graph).  The neighbour list runs in its
    static-capacity mode (capacity = margin x the warm-up pair count, device overflow flag checked by
    ``check_capacity``); the molecule count of ``reduce`` is frozen from warm-up as in inference
    capture (reference output_modules.py:27-43).  Replaces ~3k autograd-issued launches per step.

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
        # no AccumulateGrad node runs inside the capture; after each replay .grad points at them
        self.opt.zero_grad(set_to_none=True)
        params = self.reduce.params
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.static_loss = self.loss(self.z, self.pos, self.batch, self.y, self.neg_dy)
            grads = torch.autograd.grad(self.static_loss, params, allow_unused=True)
        torch.cuda.synchronize(dev)
        self.static_grads = [torch.zeros_like(p) if g is None else g for p, g in zip(params, grads)]
        self.overflow = rep.distance.last_overflow

    def step(self, z=None, pos=None, batch=None, y=None, neg_dy=None):
        with torch.no_grad():
            for dst, src in ((self.pos, pos), (self.y, y), (self.neg_dy, neg_dy)):
                if src is not None:
                    dst.copy_(src)
        self.graph.replay()
        for p, g in zip(self.reduce.params, self.static_grads):
            p.grad = g
        self.reduce()
        if self.lr_warmup_steps and self.global_step < self.lr_warmup_steps:
            scale = min(1.0, float(self.global_step + 1) / float(self.lr_warmup_steps))
            for g in self.opt.param_groups:
                g["lr"] = scale * self.lr
        self.opt.step()
        self.global_step += 1
        return self.static_loss.detach()

    def check_capacity(self):
        if bool(self.overflow.item()):
            raise RuntimeError(f"neighbour pairs exceed the captured edge capacity {self.edge_capacity}")

    def release(self):
        for d in self.dists:
            d.static_capacity = None
