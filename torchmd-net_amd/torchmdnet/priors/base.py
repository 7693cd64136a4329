"""Prior base class (reference torchmdnet/priors/base.py)."""
from typing import Dict, Optional

from torch import Tensor, nn


class BasePrior(nn.Module):
    def __init__(self, dataset=None):
        super().__init__()

    def get_init_args(self):
        return {}

    def pre_reduce(self, x, z, pos, batch, extra_args: Optional[Dict[str, Tensor]]):
        return x

    def post_reduce(self, y, z, pos, batch, extra_args: Optional[Dict[str, Tensor]]):
        return y
