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

    def step(self, z, pos, batch, y, neg_dy):
        self.opt.zero_grad(set_to_none=False)
        loss = self.loss(z, pos, batch, y, neg_dy)
        loss.backward()
        self.reduce()
        if self.lr_warmup_steps and self.global_step < self.lr_warmup_steps:
            scale = min(1.0, float(self.global_step + 1) / float(self.lr_warmup_steps))
            for g in self.opt.param_groups:
                g["lr"] = scale * self.lr
        self.opt.step()
        self.global_step += 1
        return loss.detach()
