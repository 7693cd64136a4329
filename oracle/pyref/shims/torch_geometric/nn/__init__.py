"""Minimal PyG-2.3.1 ``MessagePassing`` restatement used ONLY to execute the reference package
(/root/reference) on CPU when generating golden fixtures.  Semantics followed
(flow="source_to_target"): ``x_j = x[edge_index[0]]``, ``x_i = x[edge_index[1]]`` gathered along
``node_dim``; messages are aggregated into ``edge_index[1]`` with ``dim_size`` = number of nodes.
Pinned by the reference's own ``tests/expected.pkl`` (see tests/golden/gen_reference_fixtures.py).
"""
import inspect
import torch
from torch_scatter import scatter


class MessagePassing(torch.nn.Module):
    def __init__(self, aggr="add", node_dim=-2, **kwargs):
        super().__init__()
        self.aggr = aggr
        self.node_dim = node_dim

    def jittable(self):
        return self

    def propagate(self, edge_index, size=None, **kwargs):
        names = list(inspect.signature(self.message).parameters)
        margs = {}
        dim_size = None
        for name in names:
            if name.endswith("_i") or name.endswith("_j"):
                t = kwargs[name[:-2]]
                if t is None:
                    margs[name] = None
                    continue
                nd = self.node_dim % t.dim()
                dim_size = t.size(nd)
                idx = edge_index[1] if name.endswith("_i") else edge_index[0]
                margs[name] = t.index_select(nd, idx)
            else:
                margs[name] = kwargs[name]
        out = self.message(**margs)
        out = self.aggregate(out, edge_index[1], None, dim_size)
        return self.update(out)

    def aggregate(self, inputs, index, ptr=None, dim_size=None):
        reduce = "sum" if self.aggr == "add" else self.aggr
        return scatter(inputs, index, dim=self.node_dim, dim_size=dim_size, reduce=reduce)

    def update(self, inputs):
        return inputs
