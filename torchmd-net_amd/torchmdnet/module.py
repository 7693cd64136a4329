"""Training harness of the hot path: the reference's ``LNNP`` LightningModule
(torchmdnet/module.py:13-259) without Lightning, plus the epoch loop that replaces its Trainer.

Semantics kept from the reference: the model is ``create_model(hparams, prior, mean, std)`` or
``load_model(hparams.load_model)``; ``step`` evaluates energies and forces (forces through
``create_graph`` autograd on the positions, so the force loss trains through the double backward),
losses per stage -- train: MSE; val: L1 and MSE (the MSE drives the total); test: L1 -- weighted by
``y_weight`` / ``neg_dy_weight``, with an exponential moving average of the train/val losses when
``ema_alpha_y`` / ``ema_alpha_neg_dy`` < 1; AdamW + ReduceLROnPlateau on ``val_loss`` (epoch
interval) and a linear LR warm-up over ``lr_warmup_steps``; epoch-end mean losses keyed
``{stage}_{type}_{loss_fn}``.

MI355X: one process per GPU; the gradient average is ONE fused RCCL all-reduce per step
(``training.GradAllReduce``), the epoch-end loss means one all-reduce per epoch.
"""
from collections import defaultdict
from types import SimpleNamespace

import torch
import torch.distributed as dist
from torch.nn.functional import l1_loss, mse_loss

from . import _native
from .models.model import create_model, load_model
from .et_stack import check_pending_consumed, second_order_expected
from .training import GradAllReduce

DEFAULTS = dict(charge=False, spin=False, load_model=None, lr=4e-4, weight_decay=0.0, lr_factor=0.8,
                lr_patience=15, lr_min=1e-7, lr_metric="val_loss", lr_warmup_steps=0, ema_alpha_y=1.0,
                ema_alpha_neg_dy=1.0, y_weight=1.0, neg_dy_weight=1.0, derivative=True)


class LNNP(torch.nn.Module):
    def __init__(self, hparams, prior_model=None, mean=None, std=None):
        super().__init__()
        hp = dict(DEFAULTS)
        hp.update(vars(hparams) if isinstance(hparams, SimpleNamespace) else dict(hparams))
        self.hparams = SimpleNamespace(**hp)
        if self.hparams.load_model:
            self.model = load_model(self.hparams.load_model, args=hp)
        else:
            self.model = create_model(hp, prior_model, mean, std)
        self.global_step = 0
        self.current_epoch = 0
        self._reset_ema_dict()
        self._reset_losses_dict()

    # ---------------------------------------------------------------- optimisation
    def configure_optimizers(self):
        opt = torch.optim.AdamW(self.model.parameters(), lr=self.hparams.lr, weight_decay=self.hparams.weight_decay)
        sched = torch.optim.lr_scheduler.ReduceLROnPlateau(opt, "min", factor=self.hparams.lr_factor,
                                                           patience=self.hparams.lr_patience,
                                                           min_lr=self.hparams.lr_min)
        return opt, sched

    def optimizer_step(self, optimizer):
        """Linear warm-up of the LR over the first ``lr_warmup_steps`` steps (module.py:181-193)."""
        if self.global_step < self.hparams.lr_warmup_steps:
            scale = min(1.0, float(self.global_step + 1) / float(self.hparams.lr_warmup_steps))
            for pg in optimizer.param_groups:
                pg["lr"] = scale * self.hparams.lr
        optimizer.step()
        _native.invalidate_stack_cache()  # (a fused optimizer leaves the parameter versions unchanged)
        optimizer.zero_grad()
        self.global_step += 1

    # ---------------------------------------------------------------- forward / losses
    def forward(self, z, pos, batch=None, q=None, s=None, extra_args=None):
        return self.model(z, pos, batch=batch, q=q, s=s, extra_args=extra_args)

    def training_step(self, batch, batch_idx=0):
        return self.step(batch, [mse_loss], "train")

    def validation_step(self, batch, batch_idx=0, dataloader_idx=0):
        if dataloader_idx == 0:
            return self.step(batch, [l1_loss, mse_loss], "val")
        return self.step(batch, [l1_loss], "test")

    def test_step(self, batch, batch_idx=0):
        return self.step(batch, [l1_loss], "test")

    def _update_loss_with_ema(self, stage, kind, loss_name, loss):
        alpha = getattr(self.hparams, f"ema_alpha_{kind}")
        if stage in ("train", "val") and alpha < 1:
            ema = self.ema[stage][kind].get(loss_name, loss.detach())
            loss = alpha * loss + (1 - alpha) * ema
            self.ema[stage][kind][loss_name] = loss.detach()
        return loss

    def _compute_losses(self, y, neg_y, batch, loss_fn, stage):
        loss_y, loss_neg_y = 0.0, 0.0
        name = loss_fn.__name__
        if self.hparams.derivative and "neg_dy" in batch:
            loss_neg_y = self._update_loss_with_ema(stage, "neg_dy", name, loss_fn(neg_y, batch.neg_dy))
        if "y" in batch:
            loss_y = self._update_loss_with_ema(stage, "y", name, loss_fn(y, batch.y))
        return {"y": loss_y, "neg_dy": loss_neg_y}

    def step(self, batch, loss_fn_list, stage):
        assert len(loss_fn_list) > 0
        train_forces = stage == "train" and self.hparams.derivative and self.hparams.neg_dy_weight > 0
        with torch.set_grad_enabled(stage == "train" or self.hparams.derivative), second_order_expected(train_forces):
            extra = {k: v for k, v in batch.to_dict().items() if k not in ("y", "neg_dy", "z", "pos", "batch", "q", "s")}
            y, neg_dy = self(batch.z, batch.pos, batch=batch.batch,
                             q=batch.q if self.hparams.charge else None,
                             s=batch.s if self.hparams.spin else None, extra_args=extra)
        if self.hparams.derivative and "y" not in batch:
            neg_dy = neg_dy + y.sum() * 0
        if "y" in batch and batch.y.ndim == 1:
            batch.y = batch.y.unsqueeze(1)
        total = None
        for loss_fn in loss_fn_list:
            sl = self._compute_losses(y, neg_dy, batch, loss_fn, stage)
            name = loss_fn.__name__
            if self.hparams.neg_dy_weight > 0:
                self.losses[stage]["neg_dy"][name].append(torch.as_tensor(sl["neg_dy"]).detach())
            if self.hparams.y_weight > 0:
                self.losses[stage]["y"][name].append(torch.as_tensor(sl["y"]).detach())
            total = sl["y"] * self.hparams.y_weight + sl["neg_dy"] * self.hparams.neg_dy_weight
            self.losses[stage]["total"][name].append(torch.as_tensor(total).detach())
        return total

    # ---------------------------------------------------------------- epoch bookkeeping
    def _get_mean_loss_dict_for_type(self, kind):
        out = {}
        for stage in ("train", "val", "test"):
            for name, vals in self.losses[stage][kind].items():
                out[f"{stage}_{kind}_{name}"] = torch.stack([v.float().reshape(()) for v in vals]).mean()
        return out

    def epoch_metrics(self, group=None):
        """Epoch-end means (on_validation_epoch_end); averaged over ranks (``sync_dist=True``)."""
        res = {}
        for kind in ("total", "y", "neg_dy"):
            res.update(self._get_mean_loss_dict_for_type(kind))
        if res and dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
            keys = sorted(res)
            t = torch.stack([res[k].detach().to(torch.float64) for k in keys])
            dev = next(self.model.parameters()).device
            t = t.to(dev)
            dist.all_reduce(t, group=group)
            t /= dist.get_world_size(group)
            res = dict(zip(keys, t.cpu()))
        return {k: float(v) for k, v in res.items()}

    def _reset_losses_dict(self):
        self.losses = {s: {k: defaultdict(list) for k in ("total", "y", "neg_dy")} for s in ("train", "val", "test")}

    def _reset_ema_dict(self):
        self.ema = {s: {k: {} for k in ("y", "neg_dy")} for s in ("train", "val")}


def _val_loss(metrics):
    """Fallback monitor: the validation total of the MSE loss (the checkpoint metric of
    scripts/train.py:146)."""
    return metrics.get("val_total_mse_loss", metrics.get("val_total_l1_loss"))


def _atom_counts(dataset):
    """Atoms of every sample: the dataset's own ``atom_counts()`` when it has one (through Subset /
    FloatCast wrappers), else one pass over the samples."""
    idx = None
    ds = dataset
    while True:
        if isinstance(ds, torch.utils.data.Subset):
            idx = [ds.indices[i] for i in idx] if idx is not None else list(ds.indices)
            ds = ds.dataset
        elif hasattr(ds, "dataset") and not hasattr(ds, "atom_counts"):
            ds = ds.dataset
        else:
            break
    counts = getattr(ds, "atom_counts", None)
    if counts is not None:
        c = counts()
        return [c[i] for i in idx] if idx is not None else list(c)
    return [int(dataset[i].z.shape[0]) for i in range(len(dataset))]


def default_atom_buckets(dataset, batch_size, growth=1.125):
    """Atom capacities of the padded training batches: geometric steps (``growth``) from a little
    below the mean batch size to ``batch_size`` x the largest molecule of the dataset (every sample is
    counted: a capacity below the largest possible batch would fail mid-epoch)."""
    import math
    sizes = _atom_counts(dataset)
    mean, big = sum(sizes) / len(sizes), max(sizes)
    lo, hi = int(0.85 * mean * batch_size), big * batch_size + 1
    out, a = [], max(32, lo)
    while True:
        c = int(math.ceil(a / 32.0) * 32)
        if not out or c > out[-1]:
            out.append(c)
        if c >= hi:
            return out
        a *= growth


def fit(lnnp, datamodule, epochs, device, group=None, test_interval=0, log=None, checkpoint=None, graphed=False,
        atom_buckets=None):
    """Epoch loop replacing Lightning's Trainer + DDPStrategy (scripts/train.py:126-202): per-rank
    shards, one fused gradient all-reduce per step, LR warm-up and ReduceLROnPlateau on val_loss,
    epoch metrics averaged over ranks; rank 0 writes a Lightning-layout checkpoint
    (``{"state_dict": {"model.*": ...}, "hyper_parameters": ...}``, what ``load_model`` reads).

    ``graphed``: every training step is ONE HIP-graph replay of the force-matching step on a padded batch
    (training.PaddedGraphedTrainer; one capture per atom capacity of ``atom_buckets``, default
    ``default_atom_buckets``); the same objective, EMA, warm-up and optimiser (fused AdamW)."""
    hp = lnnp.hparams
    if graphed:
        from .training import PaddedBatches, PaddedGraphedTrainer
        bs = datamodule.hparams["batch_size"]
        if atom_buckets is None:
            atom_buckets = default_atom_buckets(datamodule.train_dataset, bs)
        rep = lnnp.model.representation_model
        batches = PaddedBatches(atom_buckets, bs, float(rep.cutoff_upper))
        trainer = PaddedGraphedTrainer(lnnp.model, batches, lr=hp.lr, weight_decay=hp.weight_decay,
                                       y_weight=hp.y_weight, neg_dy_weight=hp.neg_dy_weight if hp.derivative else 0.0,
                                       ema_alpha_y=hp.ema_alpha_y, ema_alpha_neg_dy=hp.ema_alpha_neg_dy,
                                       lr_warmup_steps=hp.lr_warmup_steps, group=group)
        opt = trainer.opt
        sched = torch.optim.lr_scheduler.ReduceLROnPlateau(opt, "min", factor=hp.lr_factor, patience=hp.lr_patience,
                                                           min_lr=hp.lr_min)
        lnnp.graphed_trainer = trainer
    else:
        opt, sched = lnnp.configure_optimizers()
        reduce = GradAllReduce(lnnp.model.parameters(), group)
    history = []
    for epoch in range(epochs):
        lnnp.current_epoch = epoch
        train = datamodule.loader("train", batches.collate if graphed else None)
        train.sampler.set_epoch(epoch)
        lnnp.model.train()
        for i, b in enumerate(train):
            if graphed:
                ly, lf, total = trainer.step(b)
                for kind, v in (("y", ly), ("neg_dy", lf)):
                    if getattr(hp, f"{kind}_weight") > 0:
                        lnnp.losses["train"][kind]["mse_loss"].append(v.detach())
                lnnp.losses["train"]["total"]["mse_loss"].append(total.detach())
                lnnp.global_step = trainer.global_step
                continue
            b = b.to(device, non_blocking=True)
            loss = lnnp.training_step(b, i)
            params = reduce.params
            loss.backward(inputs=params)
            check_pending_consumed()
            reduce()
            lnnp.optimizer_step(opt)
        if graphed:
            trainer.finish()
        lnnp.model.eval()
        for i, b in enumerate(datamodule.loader("val")):
            lnnp.validation_step(b.to(device, non_blocking=True), i, 0)
        if test_interval > 0 and epoch > 0 and epoch % test_interval == 0 and len(datamodule.test_dataset):
            for i, b in enumerate(datamodule.loader("test")):
                lnnp.validation_step(b.to(device, non_blocking=True), i, 1)
        m = lnnp.epoch_metrics(group)
        m["epoch"] = float(epoch)
        m["lr"] = opt.param_groups[0]["lr"]
        vl = m.get(lnnp.hparams.lr_metric, _val_loss(m))  # the scheduler's monitor (module.py:55)
        if vl is not None:
            sched.step(vl)
        lnnp._reset_losses_dict()
        history.append(m)
        if log is not None:
            log(m)
        rank0 = not (dist.is_available() and dist.is_initialized()) or dist.get_rank(group) == 0
        if checkpoint is not None and rank0:
            save_checkpoint(lnnp, checkpoint, epoch)
    return history


def save_checkpoint(lnnp, path, epoch=0):
    sd = {"model." + k: v.detach().cpu() for k, v in lnnp.model.state_dict().items()}
    torch.save({"state_dict": sd, "hyper_parameters": dict(vars(lnnp.hparams)), "epoch": epoch}, path)
