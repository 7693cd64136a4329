"""Graph-replayed ET-QM9 energy+force steps (the bench workload) bracketed by marker kernels, for
rocprofv3 --kernel-trace (tools/trace_summary.py lists the kernels of the marked replay).
usage: graph_trace.py [et|tn|train|tn_train|tn_c5]   (train / tn_train: the replay of the captured ET-QM9 /
TensorNet-rMD17 C3 training step; tn_c5: one EAGER TensorNet energy+force evaluation of the C5 water box)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "torchmd-net_amd"), ROOT]
import torch  # noqa: E402
import yaml  # noqa: E402

from bench import et_args, qm9_like  # noqa: E402
from torchmdnet.graphs import GraphedEnergyForces  # noqa: E402
from torchmdnet.models.model import create_model  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
which = sys.argv[1] if len(sys.argv) > 1 else "et"
if which == "tn_c5":
    import bench
    model, z, pos, batch, _ = bench.tn_water_box_model(50001, True, 0, dev)
    for _ in range(2):
        model(z, pos, batch)
    torch.cuda.synchronize()
    torch.cuda._sleep(100)
    model(z, pos, batch)
    torch.cuda._sleep(100)
    torch.cuda.synchronize()
    sys.exit(0)
if which in ("et", "train"):
    model = create_model(et_args(128)).to(dev)
    z, pos, batch = qm9_like(32, 1)
else:  # tn, tn_train: TensorNet-rMD17 (C3)
    from bench import rmd17_like
    with open(os.path.join(ROOT, "tests", "golden", "configs", "tensornet_rmd17.yaml")) as f:
        args = yaml.safe_load(f)
    args.update(prior_model=None, precision=32, derivative=True)
    model = create_model(args).to(dev)
    z, pos, batch = rmd17_like(8, 1)
z, pos, batch = z.to(dev), pos.float().to(dev), batch.to(dev)
if which in ("train", "tn_train"):
    from torchmdnet.training import GraphedTrainStep
    g = torch.Generator().manual_seed(200)
    y_lab = torch.randn(int(batch.max()) + 1, 1, generator=g).to(dev)
    f_lab = torch.randn(z.shape[0], 3, generator=g).to(dev)
    tr = GraphedTrainStep(model, z, pos, batch, y_lab, f_lab, lr=1e-4)
    for _ in range(3):
        tr.graph.replay()
    torch.cuda.synchronize()
    torch.cuda._sleep(100)
    tr.graph.replay()
    torch.cuda._sleep(100)
    torch.cuda.synchronize()
    tr.release()
    sys.exit(0)
gm = GraphedEnergyForces(model, z, pos, batch)
for _ in range(5):
    gm(pos)
torch.cuda.synchronize()
torch.cuda._sleep(100)
gm(pos)
torch.cuda._sleep(100)
torch.cuda.synchronize()
gm.release()
