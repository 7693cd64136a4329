"""Reference torchmdnet/datasets/custom.py:7-116: coordinates / atom types / energies / forces from
NumPy files matched by glob patterns (sorted), one sample per frame.  Frames are read through
memory maps (``mmap_mode="r"``), so a multi-GB coordinate file is never loaded whole."""
import glob

import numpy as np
import torch

from ..data import Data


class Custom(torch.utils.data.Dataset):
    def __init__(self, coordglob, embedglob, energyglob=None, forceglob=None):
        if energyglob is None and forceglob is None:
            raise AssertionError("Either energies, forces or both must be specified as the target")
        self.has_energies = energyglob is not None
        self.has_forces = forceglob is not None
        self.coordfiles = sorted(glob.glob(coordglob))
        self.embedfiles = sorted(glob.glob(embedglob))
        self.energyfiles = sorted(glob.glob(energyglob)) if self.has_energies else None
        self.forcefiles = sorted(glob.glob(forceglob)) if self.has_forces else None
        n = len(self.coordfiles)
        for name, files in (("embed", self.embedfiles), ("energy", self.energyfiles), ("force", self.forcefiles)):
            if files is not None and len(files) != n:
                raise AssertionError(f"Number of coordinate files {n} does not match number of {name} files "
                                     f"{len(files)}.")
        self.index = []
        self._n_atoms = []  # atoms per file group (every frame of a group has the same atoms)
        for i in range(n):
            coords = np.load(self.coordfiles[i], mmap_mode="r")
            embed = np.load(self.embedfiles[i])
            if coords.shape[1] != embed.shape[0]:
                raise AssertionError(f"Number of atoms in coordinate file {i} ({coords.shape[1]}) does not match "
                                     f"number of atoms in embed file {i} ({embed.shape[0]}).")
            if self.has_energies:
                en = np.load(self.energyfiles[i], mmap_mode="r")
                if en.shape[0] != coords.shape[0]:
                    raise AssertionError(f"Number of frames in coordinate file {i} ({coords.shape[0]}) does not "
                                         f"match number of frames in energy file {i} ({en.shape[0]}).")
            if self.has_forces:
                fo = np.load(self.forcefiles[i], mmap_mode="r")
                if fo.shape != coords.shape:
                    raise AssertionError(f"Data shape of coordinate file {i} {coords.shape} does not match the "
                                         f"shape of force file {i} {fo.shape}.")
            self.index.extend((i, k) for k in range(coords.shape[0]))
            self._n_atoms.append(int(embed.shape[0]))

    def __len__(self):
        return len(self.index)

    # open file groups kept per process (memory maps duplicate their file descriptor: a dataset of
    # thousands of groups must not hold them all open)
    MAX_OPEN_GROUPS = 64

    def atom_counts(self):
        """Atoms of every sample, without opening any sample (default_atom_buckets)."""
        return [self._n_atoms[f] for f, _ in self.index]

    def _file(self, f):
        """The memory maps / atom types of file group f, opened once per process (the loader's worker
        processes each open their own on first use) and kept in a small LRU: a sample costs a few array
        copies, not four file opens."""
        from collections import OrderedDict
        mm = self.__dict__.get("_mm")
        if mm is None:
            mm = self.__dict__["_mm"] = OrderedDict()
        if f in mm:
            mm.move_to_end(f)
            return mm[f]
        while len(mm) >= self.MAX_OPEN_GROUPS:
            mm.popitem(last=False)
        mm[f] = (np.load(self.coordfiles[f], mmap_mode="r"),
                 torch.from_numpy(np.load(self.embedfiles[f]).astype(np.int64)),
                 np.load(self.energyfiles[f], mmap_mode="r") if self.has_energies else None,
                 np.load(self.forcefiles[f], mmap_mode="r") if self.has_forces else None)
        return mm[f]

    def __getstate__(self):  # memory maps are per process
        st = dict(self.__dict__)
        st.pop("_mm", None)
        return st

    def __getitem__(self, idx):
        f, k = self.index[idx]
        coords, z, en, fo = self._file(f)
        d = Data(pos=torch.from_numpy(np.array(coords[k])), z=z.clone())
        if self.has_energies:
            d.y = torch.from_numpy(np.array(en[k]))
        if self.has_forces:
            d.neg_dy = torch.from_numpy(np.array(fo[k]))
        return d
