"""One rank of tests/test_gpu_multirank.py (launched by torch.distributed.run; every rank on cuda:0,
gloo -- RCCL refuses two ranks on one device).  The data-parallel training step of SURVEY.md 8(e) on
the real model: ET-SPICE (C4 shapes), GraphedTrainStep (forward + force pass + double backward in one
HIP graph per rank), one fused all-reduce of the flat gradient, fused AdamW -- the path the reference
runs as Lightning DDP over NCCL (scripts/train.py:175-189).

Each rank starts from ITS OWN random initial weights and its own molecules; the checks:
1. after the trainer's construction every rank holds rank 0's initial weights (broadcast);
2. the first replay's all-reduced gradient equals the mean over ranks of the eager single-rank
   gradients (LNNPStep on the same weights, no collective);
3. after 5 steps the replicas are bit-identical.
Writes a JSON verdict to argv[1] (rank 0)."""
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torchmd-net_amd"))


def flat(ts):
    return torch.cat([t.detach().reshape(-1) for t in ts])


def main(out_path):
    import yaml
    from torchmdnet.models.model import create_model
    from torchmdnet.training import GraphedTrainStep, LNNPStep
    rank, ws = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    dev = torch.device("cuda", 0)
    with open(os.path.join(ROOT, "tests", "golden", "configs", "et_spice.yaml")) as f:
        args = yaml.safe_load(f)
    args.update(prior_model=None, precision=32, derivative=True, output_model="Scalar")
    torch.manual_seed(10 + rank)  # different initial weights on every rank
    model = create_model(args).to(dev)
    params = [p for p in model.parameters() if p.requires_grad]
    w_rank0 = flat(params).clone()
    dist.broadcast(w_rank0, 0)
    differed = torch.tensor([float(not torch.equal(flat(params), w_rank0))], device=dev)
    dist.all_reduce(differed, op=dist.ReduceOp.MAX)  # (rank 0 compares with itself)
    differed = bool(differed.item())
    g = torch.Generator().manual_seed(1 + rank)  # different molecules on every rank
    n_mol = 16
    z = torch.randint(1, 9, (n_mol * 40,), generator=g).to(dev)
    pos = (torch.randn(n_mol * 40, 3, generator=g, dtype=torch.float64) * 2.5).float().to(dev)
    batch = torch.arange(n_mol).repeat_interleave(40).to(dev)
    y = torch.randn(n_mol, 1, generator=g).to(dev)
    f = torch.randn(n_mol * 40, 3, generator=g).to(dev)

    # eager single-rank gradient on the broadcast weights (LNNPStep broadcasts in its constructor)
    ref = LNNPStep(model, lr=0.0, y_weight=0.5, neg_dy_weight=0.5)
    got_w0 = torch.equal(flat(params), w_rank0)
    loss = ref.loss(z, pos, batch, y, f)
    g_local = flat(torch.autograd.grad(loss, params)).clone()
    del loss, ref
    g_all = [torch.empty_like(g_local) for _ in range(ws)]
    dist.all_gather(g_all, g_local)
    g_mean = torch.stack(g_all).mean(0)

    tr = GraphedTrainStep(model, z, pos, batch, y, f, lr=1e-3, y_weight=0.5, neg_dy_weight=0.5)
    tr.step()
    g_red = tr.reduce.flat[:-1].clone()
    grad_rel = float((g_red - g_mean).norm() / g_mean.norm())
    ranks_differ_in_grad = float((g_all[0] - g_all[-1]).norm() / g_all[0].norm())
    for _ in range(4):
        tr.step()
    tr.check_capacity()
    tr.release()
    torch.cuda.synchronize()
    w = flat(params)
    w_all = [torch.empty_like(w) for _ in range(ws)]
    dist.all_gather(w_all, w)
    identical = all(torch.equal(w_all[0], wi) for wi in w_all[1:])
    moved = float((w - w_rank0).norm() / w_rank0.norm())
    ok = torch.tensor([float(got_w0)], device=dev)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if rank == 0:
        with open(out_path, "w") as fh:
            json.dump({"world_size": ws, "initial_weights_differed": differed, "all_start_from_rank0": bool(ok.item()),
                       "reduced_grad_vs_mean_of_eager_rel": grad_rel,
                       "rank_grads_differ_rel": ranks_differ_in_grad, "replicas_identical_after_5_steps": identical,
                       "weights_moved_rel": moved, "skipped_steps": tr.skipped_steps,
                       "edge_capacity": tr.edge_capacity}, fh)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
