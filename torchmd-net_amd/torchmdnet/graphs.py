"""HIP-graph capture of the energy + force evaluation (replaces the reference's CUDA-graph path,
tests/test_model.py:87-126 / benchmarks/neighbors.py:89-99, for the ET and TensorNet models).

The reference ET is not graph-capturable (host syncs in OptimizedDistance.check_errors/resize_to_fit,
output_modules.py:33, utils.py:93).  Here the neighbour graph switches to its static-capacity mode
(no host synchronisation, padded CSR), the molecule count of ``reduce`` is frozen from a warm-up
call (the reference's own capture rule, output_modules.py:27-43), and one HIP graph replays the
whole forward + autograd force pass: ~600 launches become one graph launch.

    gm = GraphedEnergyForces(model, z, pos, batch)      # warm-up + capture
    y, neg_dy = gm(pos_new)                              # copy-in + replay (same z/batch layout)
    gm.check_capacity()                                  # raises if a replay overflowed capacity
"""
import math

import torch


def _distance_modules(model):
    from .models.utils import OptimizedDistance
    return [m for m in model.modules() if isinstance(m, OptimizedDistance)]


class GraphedEnergyForces:
    def __init__(self, model, z, pos, batch, edge_capacity=None, margin=1.25, warmup=3):
        if not model.derivative:
            raise ValueError("GraphedEnergyForces captures TorchMD_Net(derivative=True)")
        rep = model.representation_model
        self.model = model
        dev = pos.device
        self.z = z.clone()
        self.batch = batch.clone()
        self.pos = pos.detach().clone()
        # eager warm-up: sizes the edge capacity and the molecule count
        y, f = model(self.z, self.pos.clone(), self.batch)
        dists = _distance_modules(model)
        if edge_capacity is None:
            from .models.utils import OptimizedDistance  # noqa: F401
            g = rep.distance.graph(self.pos, self.batch)
            edge_capacity = int(math.ceil(g.num_pairs * margin / 256.0) * 256)
        self.edge_capacity = int(edge_capacity)
        for d in dists:
            d.static_capacity = self.edge_capacity
        self.pos.requires_grad_(True)
        try:  # pos is a leaf created outside the capture stream; its AccumulateGrad is never used
            torch.autograd.graph.set_warn_on_accumulate_grad_stream_mismatch(False)
        except AttributeError:
            pass
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                model(self.z, self.pos, self.batch)
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize(dev)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, capture_error_mode="thread_local"):
            self.y, self.neg_dy = model(self.z, self.pos, self.batch)
        torch.cuda.synchronize(dev)
        # device flag written by every replay (lives in the graph's memory pool)
        self.overflow = rep.distance.last_overflow
        self.dists = dists

    def __call__(self, pos=None):
        if pos is not None:
            with torch.no_grad():
                self.pos.copy_(pos)
        self.graph.replay()
        return self.y, self.neg_dy

    def check_capacity(self):
        """Host check (synchronises): the last replay's neighbour list fit the static capacity."""
        if bool(self.overflow.item()):
            raise RuntimeError(f"neighbour pairs exceed the captured edge capacity {self.edge_capacity}")

    def release(self):
        for d in self.dists:
            d.static_capacity = None
