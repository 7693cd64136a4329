"""Reference torchmdnet/datasets/hdf.py:7-86: ';'-separated HDF5 files; every group (except
``_metadata``, whose arrays become dataset attributes) holds per-conformation arrays ``types``
(n_conf, n_atoms), ``pos`` (n_conf, n_atoms, 3), ``energy`` (n_conf) and optionally ``forces``
(n_conf, n_atoms, 3) and ``partial_charges``.  1-D fields come out as [[value]] (the reference's
``y`` shape).  Needs ``h5py``, which this image lacks: constructing the dataset then raises
ImportError; the format logic is tested through ``_opener`` with an in-memory stand-in of the h5py
File interface (files are opened lazily per process, as the reference does)."""
import numpy as np
import torch

from ..data import Data


def _h5_open(path):
    try:
        import h5py
    except ImportError as e:  # pragma: no cover - image without h5py
        raise ImportError("torchmdnet.datasets.HDF5 needs h5py") from e
    return h5py.File(path, "r")


class HDF5(torch.utils.data.Dataset):
    def __init__(self, filename, _opener=None, **kwargs):
        self.filename = filename
        self._open = _opener or _h5_open
        self.index = None
        self.fields = None
        self.num_molecules = 0
        for path in filename.split(";"):
            f = self._open(path)
            for gname in f:
                g = f[gname]
                if gname == "_metadata":
                    for name in g:
                        setattr(self, name, torch.tensor(np.array(g[name])))
                    continue
                self.num_molecules += len(g["energy"])
                if self.fields is None:
                    self.fields = [("pos", "pos", torch.float32), ("z", "types", torch.long),
                                   ("y", "energy", torch.float32)]
                    if "forces" in g:
                        self.fields.append(("neg_dy", "forces", torch.float32))
                    if "partial_charges" in g:
                        self.fields.append(("partial_charges", "partial_charges", torch.float32))
            if hasattr(f, "close"):
                f.close()

    def _setup_index(self):
        self.index = []
        for path in self.filename.split(";"):
            f = self._open(path)
            for gname in f:
                if gname == "_metadata":
                    continue
                g = f[gname]
                arrays = tuple(g[key] for _, key, _ in self.fields)
                self.index.extend(arrays + (i,) for i in range(len(g["energy"])))
        if len(self.index) != self.num_molecules:
            raise AssertionError("Mismatch between previously calculated molecule count and actual molecule count")

    def __len__(self):
        return self.num_molecules

    def atom_counts(self):
        """Atoms of every sample from each group's ``types`` SHAPE (n_conf, n_atoms) -- no array is read
        (module.default_atom_buckets would otherwise load every conformation at training start)."""
        out = []
        for path in self.filename.split(";"):
            f = self._open(path)
            for gname in f:
                if gname == "_metadata":
                    continue
                g = f[gname]
                shape = tuple(g["types"].shape) if hasattr(g["types"], "shape") else np.shape(g["types"])
                out.extend([int(shape[-1])] * len(g["energy"]))
            if hasattr(f, "close"):
                f.close()
        return out

    def __getitem__(self, idx):
        if self.index is None:
            self._setup_index()
        entry = self.index[idx]
        i = entry[-1]
        d = Data()
        for (attr, _, dt), arr in zip(self.fields, entry[:-1]):
            if np.ndim(arr) == 1:
                setattr(d, attr, torch.tensor([[arr[i]]], dtype=dt))
            else:
                setattr(d, attr, torch.from_numpy(np.asarray(arr[i])).to(dt))
        return d
