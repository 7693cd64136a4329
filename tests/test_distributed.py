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
    out.put((rank, local, reduced, float(t)))
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
        assert torch.allclose(ra, mean, atol=1e-6)
        assert torch.allclose(rb, mean, atol=1e-6)
    assert m0 == m1 == 2.0
