"""On-disk dataset formats feeding the hot path: the reference's Custom NumPy
format and its HDF5 format.  Samples are ``torchmdnet.data.Data`` records (z, pos, y, neg_dy)."""
from .custom import Custom
from .hdf import HDF5

__all__ = ["Custom", "HDF5"]
