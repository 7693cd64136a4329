"""Multi-process (gloo, world_size 2, CPU) tests of the data-parallel training plumbing:
the fused gradient all-reduce equals the mean of the per-rank gradients, and bench.py's timing
helpers reduce with MAX."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from torchmdnet.training import GradAllReduce
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.SiLU(), torch.nn.Linear(16, 1))
    g = torch.Generator().manual_seed(100 + rank)
    x = torch.randn(32, 8, generator=g)
    model(x).pow(2).sum().backward()
    local = [p.grad.clone() for p in model.parameters()]
    GradAllReduce(model.parameters())()
    reduced = [p.grad.clone() for p in model.parameters()]
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    # plain numpy: a torch tensor would travel as a shared fd that dies with this process
    out.put((rank, [g.numpy() for g in local], [g.numpy() for g in reduced], float(t)))
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_grad_allreduce_is_mean_of_ranks():
    import sys
    from conftest import PKG
    sys.path.insert(0, PKG)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (l, red, m)) for r, l, red, m in (q.get(timeout=100) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (l0, r0, m0), (l1, r1, m1) = res[0], res[1]
    for a, b, ra, rb in zip(l0, l1, r0, r1):
        mean = (a + b) / 2
        assert abs(ra - mean).max() <= 1e-6
        assert abs(rb - mean).max() <= 1e-6
    assert m0 == m1 == 2.0


class _ToyPotential(torch.nn.Module):
    """Energy + forces with the TorchMD_Net.forward contract (y [B,1], neg_dy [N,3], forces through
    create_graph autograd), small enough for CPU ranks."""

    def __init__(self):
        super().__init__()
        self.emb = torch.nn.Embedding(10, 8)
        self.mlp = torch.nn.Sequential(torch.nn.Linear(11, 16), torch.nn.SiLU(), torch.nn.Linear(16, 1))

    def forward(self, z, pos, batch):
        pos = pos.requires_grad_(True) if not pos.requires_grad else pos
        h = torch.cat([self.emb(z), pos.pow(2)], dim=1)
        x = self.mlp(h)
        y = torch.zeros(int(batch.max()) + 1, 1, dtype=x.dtype).index_add(0, batch, x)
        (dy,) = torch.autograd.grad(y.sum(), pos, create_graph=True)
        return y, -dy


def _train_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from torchmdnet.training import LNNPStep
    torch.manual_seed(100 + rank)  # DIFFERENT initial weights on every rank
    model = _ToyPotential()
    init = [p.detach().clone() for p in model.parameters()]
    trainer = LNNPStep(model, lr=1e-2, lr_warmup_steps=3)  # broadcasts rank 0's weights
    after_bcast = [p.detach().clone() for p in model.parameters()]
    views_ok = all(p.grad is not None and p.grad.data_ptr() == v.data_ptr()
                   for p, v in zip(trainer.reduce.params, trainer.reduce.views))
    g = torch.Generator().manual_seed(7 + rank)  # every rank its own molecules
    losses = []
    for _ in range(5):
        z = torch.randint(1, 10, (12,), generator=g)
        pos = torch.randn(12, 3, generator=g)
        batch = torch.arange(3).repeat_interleave(4)
        y = torch.randn(3, generator=g)  # 1-D labels: unsqueezed like reference module.py:147-148
        f = torch.randn(12, 3, generator=g)
        losses.append(float(trainer.step(z, pos, batch, y, f)))
    final = [p.detach().clone() for p in model.parameters()]
    npy = lambda ts: [t.numpy() for t in ts]  # by value: the rank may exit before the parent reads
    out.put((rank, npy(init), npy(after_bcast), npy(final), views_ok, losses, trainer.opt.param_groups[0]["lr"]))
    dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_lnnp_step_broadcasts_and_keeps_replicas_identical():
    """DDP semantics (reference scripts/train.py:175-189): rank 1 starts from different weights, the
    trainer broadcasts rank 0's, every step averages the gradients in one all-reduce over the flat
    buffer the .grad tensors are views of, so the replicas stay bit-identical while training on
    disjoint data."""
    import sys
    from conftest import PKG
    sys.path.insert(0, PKG)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_train_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: rest for r, *rest in (q.get(timeout=160) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (i0, b0, f0, v0, l0, lr0), (i1, b1, f1, v1, l1, lr1) = res[0], res[1]
    eq = lambda x, y: all((a == b).all() for a, b in zip(x, y))
    assert not eq(i0, i1)  # started different
    assert eq(b0, b1)  # broadcast
    assert eq(b0, i0)  # ... of rank 0's weights
    assert eq(f0, f1)  # identical after 5 steps
    assert not eq(f0, b0)  # and they did train
    assert v0 and v1
    assert l0 != l1  # on different data
    assert lr0 == lr1 == pytest.approx(1e-2)  # warm-up over 3 steps reached the base LR


def _split_model(kind):
    if kind == "last_largest":  # the last parameter holds most elements: the TAIL bucket is empty
        return torch.nn.Sequential(torch.nn.Linear(8, 4), torch.nn.SiLU(), torch.nn.Linear(4, 300, bias=False))
    return torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.SiLU(), torch.nn.Linear(16, 4), torch.nn.Linear(4, 1))


def _split_worker(rank, world, port, out, kind="balanced"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from torchmdnet.training import GradAllReduce, SplitAdamW, _adamw, step_reduce
    torch.manual_seed(0)
    model = _split_model(kind)
    ref = _split_model(kind)
    ref.load_state_dict(model.state_dict())
    red = GradAllReduce(model.parameters())
    tail, head = red.split_params()
    opt = SplitAdamW(tail, head, 1e-2, 0.01)
    red_ref = GradAllReduce(ref.parameters())
    opt_ref = _adamw(red_ref.params, 1e-2, 0.01)
    seen = []
    g = torch.Generator().manual_seed(100 + rank)
    for _ in range(3):
        x = torch.randn(32, 8, generator=g)
        for m in (model, ref):
            m.zero_grad(set_to_none=False)
            m(x).pow(2).sum().backward()
        # the tail bucket (last parameters + the skip flag) is averaged before the first part steps
        step_reduce(red, opt, lambda: seen.append(float(red.flag[0])))
        red_ref()
        opt_ref.step()
    same = all(torch.equal(p, q) for p, q in zip(model.parameters(), ref.parameters()))
    both = (len(tail) > 0 and len(head) > 0) if kind == "balanced" else (len(tail) == 0 and len(head) > 0)
    out.put((rank, same, both, seen, [p.detach().numpy() for p in model.parameters()]))
    dist.destroy_process_group()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("kind", ["balanced", "last_largest"])
def test_two_bucket_allreduce_overlapped_step_equals_fused(kind):
    """The two-bucket all-reduce with the tail bucket's AdamW update issued before the head bucket is
    reduced (training.step_reduce / SplitAdamW, world > 1) gives the SAME parameters as one fused
    all-reduce + one AdamW, on every rank (replicas identical).  ``last_largest``: the last parameter holds
    more than half of all elements, so the tail bucket is empty (the head optimizer must keep its
    slot and step only after the head bucket is averaged)."""
    import sys
    from conftest import PKG
    sys.path.insert(0, PKG)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_split_worker, args=(r, 2, port, q, kind)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: rest for r, *rest in (q.get(timeout=100) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in (0, 1):
        same, both, seen, _ = res[r]
        assert same and both and seen == [0.0, 0.0, 0.0]
    assert all((a == b).all() for a, b in zip(res[0][3], res[1][3]))
