"""Per-element energy offsets (interface of the reference's Atomref prior, torchmdnet/priors/atomref.py:8-42;
ET-QM9 uses it, examples/ET-QM9.yaml:45).

The offsets live in a one-column embedding table ``atomref`` indexed by atomic number; the values it
starts from are kept as the ``initial_atomref`` buffer (both names are state_dict keys that reference
checkpoints carry).  The table is added to the per-atom head output before the molecular sum."""
import warnings
from typing import Dict, Optional

import torch
from torch import Tensor, nn

from .base import BasePrior

# table size when a dataset has no offsets for its target (atomic numbers 0 .. 99)
_DEFAULT_ELEMENTS = 100


def _offset_table(max_z, dataset) -> Tensor:
    """The initial (n_elements, 1) offset column from a dataset, else zeros for ``max_z`` elements."""
    if dataset is not None:
        table = dataset.get_atomref()
        if table is None:
            warnings.warn(f"dataset.get_atomref() gave None (no per-element offsets for this target); "
                          f"the Atomref prior starts from zeros for {_DEFAULT_ELEMENTS} elements")
            table = torch.zeros(_DEFAULT_ELEMENTS, 1)
    elif max_z is not None:
        table = torch.zeros(max_z, 1)
    else:
        raise ValueError("Atomref prior: pass max_z or a dataset (both were None)")
    return table.reshape(-1, 1) if table.dim() == 1 else table


class Atomref(BasePrior):
    def __init__(self, max_z=None, dataset=None):
        super().__init__()
        table = _offset_table(max_z, dataset)
        self.register_buffer("initial_atomref", table)
        # the embedding's own init draws from the RNG: kept, so seeded parameter streams line up with the
        # reference's; its weights are then overwritten by the initial table
        self.atomref = nn.Embedding(table.shape[0], 1)
        self.reset_parameters()

    def reset_parameters(self):
        with torch.no_grad():
            self.atomref.weight.copy_(self.initial_atomref)

    def get_init_args(self):
        return {"max_z": int(self.initial_atomref.shape[0])}

    def pre_reduce(self, x: Tensor, z: Tensor, pos: Tensor, batch: Tensor,
                   extra_args: Optional[Dict[str, Tensor]]):
        return x + self.atomref.weight.index_select(0, z)
