"""Priors on the hot path: Atomref only (D2 / ZBL / Coulomb use torch_cluster, out of scope)."""
from .atomref import Atomref
from .base import BasePrior

__all__ = ["Atomref"]
