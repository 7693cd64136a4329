"""``torchmdnet_neighbors::get_neighbor_pairs`` -- the reference's native op, same schema.

Reference: torchmdnet/neighbors/neighbors.cpp:3-5 (schema), neighbors/__init__.py:1-17 (loader),
neighbors_cuda.cu:25-89 (CUDA + AutogradCUDA registration).  As in the reference, the op lives in a
native library loaded with ``torch.ops.load_library``: ``lib/libtmdnet_torch.so``
(``csrc/torch_ops.cpp``) registers it with ``TORCH_LIBRARY`` on the CUDA (= HIP on ROCm),
AutogradCUDA and CPU keys -- so TorchScript and libtorch (C++) consumers see it without Python --
and its compute is the HIP library (``tmdnet_nl_build``; backward ``tmdnet_nl_backward_edges``, a
HIP kernel, differentiable again).  Returned values, as in the reference: (neighbors int32 [2, P],
deltas [P, 3], distances [P], num_pairs int32 [1]) with P = max_num_pairs, padded with (-1, -1)/0.

The CPU kernel raises: there is no CPU implementation of the hot path.
"""
import torch

from .. import _native as nat

nat.load_torch_ops()
get_neighbor_pairs_kernel = torch.ops.torchmdnet_neighbors.get_neighbor_pairs

try:  # reference neighbors/__init__.py:15-17
    import torch._dynamo as dynamo
    dynamo.disallow_in_graph(get_neighbor_pairs_kernel)
except Exception:  # pragma: no cover
    pass
