"""Package utilities.

``atomic_masses``: standard atomic weights (IUPAC 2013 table, index = atomic number, index 0 = 1.0
placeholder) used by the dipole / spatial-extent output heads (same data as reference
torchmdnet/utils.py ``atomic_masses``).
"""
import numpy as np

atomic_masses = np.array([
    1.0, 1.008, 4.002602, 6.94, 9.0121831, 10.81, 12.011, 14.007,
    15.999, 18.998403163, 20.1797, 22.98976928, 24.305, 26.9815385, 28.085, 30.973761998,
    32.06, 35.45, 39.948, 39.0983, 40.078, 44.955908, 47.867, 50.9415,
    51.9961, 54.938044, 55.845, 58.933194, 58.6934, 63.546, 65.38, 69.723,
    72.63, 74.921595, 78.971, 79.904, 83.798, 85.4678, 87.62, 88.90584,
    91.224, 92.90637, 95.95, 97.90721, 101.07, 102.9055, 106.42, 107.8682,
    112.414, 114.818, 118.71, 121.76, 127.6, 126.90447, 131.293, 132.90545196,
    137.327, 138.90547, 140.116, 140.90766, 144.242, 144.91276, 150.36, 151.964,
    157.25, 158.92535, 162.5, 164.93033, 167.259, 168.93422, 173.054, 174.9668,
    178.49, 180.94788, 183.84, 186.207, 190.23, 192.217, 195.084, 196.966569,
    200.592, 204.38, 207.2, 208.9804, 208.98243, 209.98715, 222.01758, 223.01974,
    226.02541, 227.02775, 232.0377, 231.03588, 238.02891, 237.04817, 244.06421, 243.06138,
    247.07035, 247.07031, 251.07959, 252.083, 257.09511, 258.09843, 259.101, 262.11,
    267.122, 268.126, 271.134, 270.133, 269.1338, 278.156, 281.165, 281.166,
    285.177, 286.182, 289.19, 289.194, 293.204, 293.208, 294.214,
])


class MissingEnergyException(Exception):
    pass


def train_val_test_split(dset_len, train_size, val_size, test_size, seed, order=None):
    """Reference torchmdnet/utils.py:54-116: sizes as counts or fractions (one may be None = the
    rest), a seeded numpy permutation (``np.random.default_rng(seed)``), or a fixed ``order``."""
    sizes = [train_size, val_size, test_size]
    if sum(s is None for s in sizes) > 1:
        raise AssertionError("Only one of train_size, val_size, test_size is allowed to be None.")
    is_float = [isinstance(s, float) for s in sizes]
    sizes = [round(dset_len * s) if f else s for s, f in zip(sizes, is_float)]
    if None in sizes:
        k = sizes.index(None)
        sizes[k] = dset_len - sum(s for s in sizes if s is not None)
    if sum(sizes) > dset_len:  # rounding overshoot: take one from the last fractional split
        for k in (2, 1, 0):
            if is_float[k]:
                sizes[k] -= 1
                break
    train_size, val_size, test_size = sizes
    if min(sizes) < 0:
        raise AssertionError(f"One of training ({train_size}), validation ({val_size}) or testing "
                             f"({test_size}) splits ended up with a negative size.")
    total = sum(sizes)
    if dset_len < total:
        raise AssertionError(f"The dataset ({dset_len}) is smaller than the combined split sizes ({total}).")
    if total < dset_len:
        import warnings
        warnings.warn(f"{dset_len - total} samples were excluded from the dataset")
    idxs = np.arange(dset_len, dtype=int)
    if order is None:
        idxs = np.random.default_rng(seed).permutation(idxs)
    parts = [idxs[:train_size], idxs[train_size:train_size + val_size], idxs[train_size + val_size:total]]
    if order is not None:
        parts = [[order[i] for i in p] for p in parts]
    return tuple(np.array(p) for p in parts)


def make_splits(dataset_len, train_size, val_size, test_size, seed, filename=None, splits=None, order=None):
    """Reference torchmdnet/utils.py:119-146: load ``splits`` (npz with idx_train/val/test) or draw
    them, optionally save to ``filename``; returns three int64 tensors."""
    import torch
    if splits is not None:
        s = np.load(splits)
        idx_train, idx_val, idx_test = s["idx_train"], s["idx_val"], s["idx_test"]
    else:
        idx_train, idx_val, idx_test = train_val_test_split(dataset_len, train_size, val_size, test_size,
                                                            seed, order)
    if filename is not None:
        np.savez(filename, idx_train=idx_train, idx_val=idx_val, idx_test=idx_test)
    return torch.from_numpy(idx_train), torch.from_numpy(idx_val), torch.from_numpy(idx_test)
