"""Data path feeding the hot path: sample records, molecule collation, splits and
the per-rank loaders of data-parallel training.

Reference: ``torchmdnet/data.py`` (``DataModule``: Custom / named datasets, ``FloatCastDatasetWrapper``,
``make_splits``, train / val / test loaders, ``_standardize``) over PyG's ``Data`` / ``Batch`` and
``DataLoader``.  PyG is not part of this build: a sample is a ``Data`` record, and ``collate``
concatenates per-atom fields (z, pos, neg_dy, ...) and stacks per-molecule ones (y) exactly as
PyG's ``Batch.from_data_list`` does for these attributes, adding the ``batch`` vector (molecule id of
every atom).  One process per GPU: each rank draws its own disjoint, seeded shard of every epoch
(``DistributedSampler`` semantics, the reference's Lightning DDP default), batches are collated on the
host into pinned memory and copied to HBM with non-blocking transfers.
"""
import os

import torch

from .utils import MissingEnergyException, make_splits

PER_MOLECULE = ("y",)


class Data:
    """Attribute record of one molecule (or of a collated batch); ``"y" in d`` tests presence."""

    def __init__(self, **kw):
        for k, v in kw.items():
            setattr(self, k, v)

    def keys(self):
        return [k for k, v in self.__dict__.items() if v is not None]

    def __contains__(self, key):
        return getattr(self, key, None) is not None

    def to_dict(self):
        return {k: getattr(self, k) for k in self.keys()}

    def __iter__(self):
        return iter(self.to_dict().items())

    def to(self, device, non_blocking=False):
        return Data(**{k: (v.to(device, non_blocking=non_blocking) if torch.is_tensor(v) else v)
                       for k, v in self.to_dict().items()})

    def pin_memory(self):
        return Data(**{k: (v.pin_memory() if torch.is_tensor(v) else v) for k, v in self.to_dict().items()})

    @property
    def num_graphs(self):
        return int(self.batch.max()) + 1 if "batch" in self else 1


def collate(samples):
    """PyG ``Batch.from_data_list`` for the fields of this path: per-atom tensors concatenated along
    dim 0, ``y`` (per molecule) concatenated to [B, 1]-compatible rows, ``batch`` = molecule ids."""
    out = Data()
    keys = samples[0].keys()
    for k in keys:
        vals = [getattr(s, k) for s in samples]
        if k in PER_MOLECULE:
            vals = [v.reshape(1, -1) if v.dim() <= 1 else v for v in vals]
        setattr(out, k, torch.cat(vals, dim=0))
    out.batch = torch.cat([torch.full((s.z.shape[0],), i, dtype=torch.long) for i, s in enumerate(samples)])
    return out


class FloatCast(torch.utils.data.Dataset):
    """Reference ``FloatCastDatasetWrapper`` (data.py:16-40): floating fields cast to the model dtype."""

    def __init__(self, dataset, dtype=torch.float64):
        self.dataset = dataset
        self.dtype = dtype

    def __len__(self):
        return len(self.dataset)

    def __getitem__(self, idx):
        d = self.dataset[idx]
        for k, v in d:
            if torch.is_tensor(v) and torch.is_floating_point(v):
                setattr(d, k, v.to(self.dtype))
        return d

    def __getattr__(self, name):
        if name == "dataset":
            raise AttributeError(name)
        return getattr(self.dataset, name)


class ShardSampler(torch.utils.data.Sampler):
    """Per-rank shard of a (seeded, per-epoch reshuffled) permutation: ``DistributedSampler``
    semantics -- padded to a multiple of the world size so every rank runs the same step count."""

    def __init__(self, n, rank=0, world_size=1, shuffle=True, seed=0):
        self.n, self.rank, self.ws, self.shuffle, self.seed = n, rank, world_size, shuffle, seed
        self.epoch = 0
        self.per_rank = -(-n // world_size)

    def set_epoch(self, epoch):
        self.epoch = epoch

    def __iter__(self):
        if self.shuffle:
            g = torch.Generator().manual_seed(self.seed + self.epoch)
            idx = torch.randperm(self.n, generator=g).tolist()
        else:
            idx = list(range(self.n))
        total = self.per_rank * self.ws
        idx += idx[:total - len(idx)]
        return iter(idx[self.rank:total:self.ws])

    def __len__(self):
        return self.per_rank


class DataModule:
    """Reference ``DataModule`` (data.py:43-215) without Lightning: ``setup`` builds the dataset from
    hparams (``Custom`` from coord/embed/energy/force globs, ``HDF5``, or a dataset passed in), casts
    it, draws the splits (saved to ``log_dir/splits.npz``) and optionally standardises ``y``."""

    def __init__(self, hparams, dataset=None, rank=0, world_size=1):
        self.hparams = dict(hparams)
        self.dataset = dataset
        self.rank, self.world_size = rank, world_size
        self._mean, self._std = None, None
        self._loaders = {}

    def setup(self, stage=None):
        from . import datasets
        from .models.utils import dtype_mapping
        hp = self.hparams
        if self.dataset is None:
            if hp["dataset"] == "Custom":
                self.dataset = datasets.Custom(hp["coord_files"], hp["embed_files"], hp.get("energy_files"),
                                               hp.get("force_files"))
            else:
                self.dataset = getattr(datasets, hp["dataset"])(hp["dataset_root"], **(hp.get("dataset_arg") or {}))
        self.dataset = FloatCast(self.dataset, dtype_mapping[hp.get("precision", 32)])
        log_dir = hp.get("log_dir")
        if log_dir:  # (the reference's Lightning logger creates it before the data module saves the splits)
            os.makedirs(log_dir, exist_ok=True)
        self.idx_train, self.idx_val, self.idx_test = make_splits(
            len(self.dataset), hp["train_size"], hp["val_size"], hp["test_size"], hp["seed"],
            os.path.join(log_dir, "splits.npz") if log_dir else None, hp.get("splits"))
        sub = torch.utils.data.Subset
        self.train_dataset = sub(self.dataset, self.idx_train.tolist())
        self.val_dataset = sub(self.dataset, self.idx_val.tolist())
        self.test_dataset = sub(self.dataset, self.idx_test.tolist())
        if hp.get("standardize"):
            self._standardize()

    @property
    def mean(self):
        return self._mean

    @property
    def std(self):
        return self._std

    @property
    def atomref(self):
        return self.dataset.get_atomref() if hasattr(self.dataset, "get_atomref") else None

    def loader(self, stage, collate_fn=None):
        """The stage's loader (cached); ``collate_fn`` replaces ``collate`` (e.g. the fixed-shape
        ``training.PaddedBatches.collate`` of the captured training step)."""
        key = (stage, collate_fn)
        if key in self._loaders:
            return self._loaders[key]
        ds = {"train": self.train_dataset, "val": self.val_dataset, "test": self.test_dataset}[stage]
        train = stage == "train"
        bs = self.hparams["batch_size"] if train else self.hparams.get("inference_batch_size",
                                                                       self.hparams["batch_size"])
        sampler = ShardSampler(len(ds), self.rank, self.world_size, shuffle=train, seed=self.hparams.get("seed", 0))
        dl = torch.utils.data.DataLoader(ds, batch_size=bs, sampler=sampler, collate_fn=collate_fn or collate,
                                         num_workers=self.hparams.get("num_workers", 0),
                                         pin_memory=torch.cuda.is_available())
        self._loaders[key] = dl
        return dl

    def _standardize(self):
        """Mean / std of the training energies (minus the Atomref prior when it is the prior)."""
        atomref = self.atomref if self.hparams.get("prior_model") == "Atomref" else None
        dl = torch.utils.data.DataLoader(self.train_dataset, batch_size=self.hparams.get("inference_batch_size", 64),
                                         collate_fn=collate)
        ys = []
        try:
            for b in dl:
                if "y" not in b:
                    raise MissingEnergyException()
                y = b.y.clone()
                if atomref is not None:
                    ref = torch.zeros(b.num_graphs, dtype=y.dtype).index_add(0, b.batch, atomref[b.z].view(-1).to(y.dtype))
                    y = (y.squeeze() - ref.squeeze()).clone()
                ys.append(y)
        except MissingEnergyException:
            import warnings
            warnings.warn("Standardize is true but failed to compute dataset mean and standard deviation. "
                          "Maybe the dataset only contains forces.")
            return
        ys = torch.cat(ys)
        self._mean = ys.mean(dim=0)
        self._std = ys.std(dim=0)
