"""torch_scatter 2.1.1 ``scatter`` restatement (sum/add/mean) used ONLY to run the reference on CPU
for fixture generation.  Test infrastructure, not product code."""
import torch


def scatter(src, index, dim=-1, out=None, dim_size=None, reduce="sum"):
    dim = dim % src.dim()
    if index.dim() == 1:
        shape = [1] * src.dim()
        shape[dim] = -1
        index = index.view(shape).expand_as(src)
    if dim_size is None:
        dim_size = int(index.max()) + 1 if index.numel() > 0 else 0
    size = list(src.shape)
    size[dim] = dim_size
    acc = torch.zeros(size, dtype=src.dtype, device=src.device)
    if reduce in ("sum", "add"):
        return acc.scatter_add_(dim, index, src)
    if reduce == "mean":
        s = acc.scatter_add_(dim, index, src)
        c = torch.zeros(size, dtype=src.dtype, device=src.device).scatter_add_(dim, index, torch.ones_like(src))
        return s / c.clamp(min=1)
    raise NotImplementedError(reduce)
