"""CPU tests of the training harness and data path: splits, the Custom /
HDF5 formats, collation, the LNNP loss / EMA / warm-up / plateau logic, Lightning-layout
checkpoints read back by load_model, and the data-parallel epoch loop over gloo (world_size 2).

The model's hot path needs the GPU, so the LNNP logic is exercised with a tiny CPU potential that has
the TorchMD_Net.forward signature (energies + forces by autograd); the real model runs the same
harness on the GPU (bench.py's training lines)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from torchmdnet import data as D
from torchmdnet import module as M
from torchmdnet.utils import make_splits, train_val_test_split


class TinyPotential(torch.nn.Module):
    """E = sum_atoms MLP(emb(z), |pos|^2); forces = -dE/dpos (TorchMD_Net.forward signature)."""

    def __init__(self):
        super().__init__()
        self.emb = torch.nn.Embedding(10, 8)
        self.net = torch.nn.Sequential(torch.nn.Linear(9, 16), torch.nn.SiLU(), torch.nn.Linear(16, 1))

    def forward(self, z, pos, batch=None, q=None, s=None, extra_args=None):
        pos.requires_grad_(True)
        h = torch.cat([self.emb(z), (pos ** 2).sum(1, keepdim=True)], dim=1)
        e = self.net(h)
        y = torch.zeros(int(batch.max()) + 1, 1, dtype=e.dtype).index_add(0, batch, e)
        (dy,) = torch.autograd.grad(y.sum(), pos, create_graph=True)
        return y, -dy


def _tiny_lnnp(monkeypatch, **hp):
    monkeypatch.setattr(M, "create_model", lambda args, prior=None, mean=None, std=None: TinyPotential())
    return M.LNNP(dict(hp))


def _molecules(n, seed=0):
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(n):
        k = int(torch.randint(3, 7, (1,), generator=g))
        out.append(D.Data(z=torch.randint(1, 10, (k,), generator=g), pos=torch.randn(k, 3, generator=g),
                          y=torch.randn(1, generator=g), neg_dy=torch.randn(k, 3, generator=g)))
    return out


class ListDataset(torch.utils.data.Dataset):
    def __init__(self, items):
        self.items = items

    def __len__(self):
        return len(self.items)

    def __getitem__(self, i):
        d = self.items[i]
        return D.Data(**{k: v.clone() for k, v in d.to_dict().items()})


# ----------------------------------------------------------------------------- splits
def test_splits_follow_reference_semantics(tmp_path):
    # fractions round, None takes the rest, a seeded default_rng permutation (utils.py:54-116)
    tr, va, te = train_val_test_split(100, 0.8, 0.1, None, seed=1)
    assert (len(tr), len(va), len(te)) == (80, 10, 10)
    perm = np.random.default_rng(1).permutation(np.arange(100))
    assert np.array_equal(np.concatenate([tr, va, te]), perm)
    # overshoot from rounding comes off the last fractional split
    tr, va, te = train_val_test_split(10, 0.65, 0.25, 0.15, seed=0)  # round: 6 + 2 + 2 = 10 fits
    assert (len(tr), len(va), len(te)) == (6, 2, 2)
    tr, va, te = train_val_test_split(10, 0.7, 0.25, 0.15, seed=0)  # 7 + 2 + 2 > 10: test gives one
    assert (len(tr), len(va), len(te)) == (7, 2, 1)
    with pytest.raises(AssertionError):
        train_val_test_split(10, None, None, 2, seed=0)
    f = tmp_path / "splits.npz"
    a = make_splits(50, 30, 10, 10, 3, filename=str(f))
    b = make_splits(50, None, None, None, 0, splits=str(f))
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    order = list(range(99, 49, -1))
    tr, va, te = train_val_test_split(50, 20, 20, 10, seed=0, order=order)
    assert list(tr) == order[:20]


# ----------------------------------------------------------------------------- formats
def test_custom_dataset_and_collate(tmp_path):
    rng = np.random.default_rng(0)
    for i, (nf, na) in enumerate([(4, 5), (3, 7)]):
        np.save(tmp_path / f"coord_{i}.npy", rng.normal(size=(nf, na, 3)).astype(np.float32))
        np.save(tmp_path / f"embed_{i}.npy", rng.integers(1, 9, size=na))
        np.save(tmp_path / f"energy_{i}.npy", rng.normal(size=(nf, 1)).astype(np.float32))
        np.save(tmp_path / f"forces_{i}.npy", rng.normal(size=(nf, na, 3)).astype(np.float32))
    from torchmdnet.datasets import Custom
    ds = Custom(str(tmp_path / "coord_*.npy"), str(tmp_path / "embed_*.npy"), str(tmp_path / "energy_*.npy"),
                str(tmp_path / "forces_*.npy"))
    assert len(ds) == 7
    s = ds[5]  # file 1, frame 1
    assert s.pos.shape == (7, 3) and s.z.dtype == torch.int64 and s.neg_dy.shape == (7, 3)
    assert np.allclose(s.pos.numpy(), np.load(tmp_path / "coord_1.npy")[1])
    b = D.collate([ds[0], ds[5], ds[1]])
    assert b.z.shape == (17,) and b.pos.shape == (17, 3) and b.y.shape == (3, 1)
    assert torch.equal(b.batch, torch.tensor([0] * 5 + [1] * 7 + [2] * 5))
    assert "y" in b and "q" not in b
    with pytest.raises(AssertionError):
        Custom(str(tmp_path / "coord_*.npy"), str(tmp_path / "embed_*.npy"))


def test_hdf5_format_with_stand_in_file():
    """The HDF5 layout (groups of types/pos/energy[/forces], _metadata) through an in-memory stand-in
    of h5py.File (h5py is not installed in this image)."""
    rng = np.random.default_rng(1)
    files = {
        "a.h5": {"_metadata": {"atomref": np.arange(5.0)},
                 "g3": {"types": np.array([[1, 6, 8]] * 2), "pos": rng.normal(size=(2, 3, 3)),
                        "energy": rng.normal(size=2), "forces": rng.normal(size=(2, 3, 3))}},
        "b.h5": {"g2": {"types": np.array([[1, 1]] * 3), "pos": rng.normal(size=(3, 2, 3)),
                        "energy": rng.normal(size=3), "forces": rng.normal(size=(3, 2, 3))}},
    }
    from torchmdnet.datasets import HDF5
    ds = HDF5("a.h5;b.h5", _opener=lambda p: files[p])
    assert len(ds) == 5 and torch.equal(ds.atomref, torch.arange(5.0, dtype=torch.float64))
    s = ds[3]
    assert s.z.tolist() == [1, 1] and s.y.shape == (1, 1) and s.neg_dy.shape == (2, 3)
    assert np.isclose(float(s.y), files["b.h5"]["g2"]["energy"][1], atol=1e-6)
    # atom counts from the `types` shapes, in sample order, without reading arrays
    assert ds.atom_counts() == [3, 3, 2, 2, 2] == [int(ds[i].z.shape[0]) for i in range(len(ds))]
    from torchmdnet.module import _atom_counts
    assert _atom_counts(torch.utils.data.Subset(ds, [4, 0])) == [2, 3]


# ----------------------------------------------------------------------------- LNNP logic
def test_lnnp_losses_ema_and_warmup(monkeypatch):
    lnnp = _tiny_lnnp(monkeypatch, lr=1e-2, lr_warmup_steps=4, ema_alpha_y=0.5, ema_alpha_neg_dy=1.0,
                      y_weight=0.3, neg_dy_weight=0.7)
    b = D.collate(_molecules(4))
    opt, sched = lnnp.configure_optimizers()
    l0 = lnnp.training_step(b)
    y, f = lnnp.model(b.z, b.pos, b.batch)
    mse = torch.nn.functional.mse_loss
    assert torch.allclose(l0, 0.3 * mse(y, b.y) + 0.7 * mse(f, b.neg_dy), atol=1e-6)  # EMA starts at the loss
    l0.backward()
    lnnp.optimizer_step(opt)
    assert abs(opt.param_groups[0]["lr"] - 1e-2 * 1 / 4) < 1e-12  # warm-up 1/4
    raw = mse(lnnp.model(b.z, b.pos, b.batch)[0], b.y).detach()
    prev = lnnp.ema["train"]["y"]["mse_loss"]
    lnnp.training_step(b)
    assert torch.allclose(lnnp.ema["train"]["y"]["mse_loss"], 0.5 * raw + 0.5 * prev, atol=1e-6)
    lnnp.validation_step(b, 0, 0)
    lnnp.validation_step(b, 0, 1)
    m = lnnp.epoch_metrics()
    assert {"train_total_mse_loss", "val_total_l1_loss", "val_total_mse_loss", "test_total_l1_loss",
            "val_y_mse_loss", "train_neg_dy_mse_loss"} <= set(m)
    for _ in range(4):
        lnnp.optimizer_step(opt)
    assert opt.param_groups[0]["lr"] == 1e-2


def test_fit_single_process_plateau_and_checkpoint(monkeypatch, tmp_path):
    lnnp = _tiny_lnnp(monkeypatch, lr=1e-3, lr_patience=0, lr_factor=0.5, lr_metric="val_total_mse_loss")
    dm = D.DataModule(dict(batch_size=4, inference_batch_size=8, train_size=12, val_size=4, test_size=4,
                           seed=1, precision=32, log_dir=str(tmp_path)), dataset=ListDataset(_molecules(20)))
    dm.setup()
    assert os.path.exists(tmp_path / "splits.npz")
    hist = M.fit(lnnp, dm, epochs=3, device="cpu", test_interval=1, checkpoint=str(tmp_path / "last.ckpt"))
    assert len(hist) == 3 and all("val_total_mse_loss" in h for h in hist)
    assert "test_total_l1_loss" in hist[2]
    ck = torch.load(tmp_path / "last.ckpt", weights_only=True)
    assert all(k.startswith("model.") for k in ck["state_dict"]) and ck["hyper_parameters"]["lr"] == 1e-3


def test_checkpoint_loads_into_real_model(tmp_path):
    """save_checkpoint (Lightning layout) -> models.model.load_model reproduces the state dict (f4)."""
    from conftest import yaml_args
    from torchmdnet.models.model import load_model
    args = yaml_args("equivariant-transformer", embedding_dimension=32, num_layers=2, num_rbf=16,
                     num_heads=4, derivative=True)
    torch.manual_seed(0)
    lnnp = M.LNNP(args)
    p = tmp_path / "m.ckpt"
    M.save_checkpoint(lnnp, str(p))
    m2 = load_model(str(p))
    for (k, a), (k2, b) in zip(lnnp.model.state_dict().items(), m2.state_dict().items()):
        assert k == k2 and torch.equal(a, b)


def test_standardize_mean_std():
    items = _molecules(10, seed=3)
    dm = D.DataModule(dict(batch_size=4, train_size=10, val_size=0, test_size=0, seed=0, standardize=True,
                           precision=64), dataset=ListDataset(items))
    dm.setup()
    ys = torch.stack([items[int(i)].y for i in dm.idx_train]).double()
    assert torch.allclose(dm.mean, ys.mean(0)) and torch.allclose(dm.std, ys.std(0))


# ----------------------------------------------------------------------------- data parallel
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _fit_worker(rank, world, port, out):
    import sys
    from conftest import PKG
    sys.path.insert(0, PKG)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from torchmdnet import data as D_
    from torchmdnet import module as M_
    import test_training_harness as T
    M_.create_model = lambda args, prior=None, mean=None, std=None: T.TinyPotential()
    torch.manual_seed(0)  # same initial weights on every rank
    lnnp = M_.LNNP(dict(lr=1e-3))
    dm = D_.DataModule(dict(batch_size=3, train_size=12, val_size=4, test_size=0, seed=2, precision=32),
                       dataset=T.ListDataset(T._molecules(16)), rank=rank, world_size=world)
    dm.setup()
    shard = list(iter(dm.loader("train").sampler))
    hist = M_.fit(lnnp, dm, epochs=2, device="cpu")
    flat = torch.cat([p.detach().reshape(-1) for p in lnnp.model.parameters()])
    out.put((rank, shard, flat.numpy(), hist[-1]["val_total_mse_loss"]))
    dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_fit_data_parallel_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fit_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: (s, w, v) for r, s, w, v in (q.get(timeout=150) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (s0, w0, v0), (s1, w1, v1) = res[0], res[1]
    assert not set(s0) & set(s1) and len(set(s0) | set(s1)) == 12  # disjoint shards covering the split
    assert abs(w0 - w1).max() <= 1e-6  # averaged gradients keep the replicas identical
    assert abs(v0 - v1) < 1e-9  # epoch metrics are rank-averaged


# ----------------------------------------------------------------------------- padded batches (captured fit)
def test_padded_batches_layout_and_weights():
    """training.PaddedBatches: real atoms first in molecule order, ghost atoms on the dummy molecule
    spaced beyond the cutoff, weights that turn the weighted sums into the reference's mean losses."""
    import torch
    from torchmdnet.data import Data, collate
    from torchmdnet.training import PaddedBatches, padded_losses
    g = torch.Generator().manual_seed(0)
    samples = []
    for n in (5, 9, 3):
        samples.append(Data(z=torch.randint(1, 10, (n,), generator=g), pos=torch.randn(n, 3, generator=g),
                            y=torch.randn(1, generator=g), neg_dy=torch.randn(n, 3, generator=g)))
    pb = PaddedBatches([16, 24, 32], max_molecules=4, cutoff=5.0)
    b = pb.collate(samples)
    ref = collate(samples)
    assert b.capacity == 24 and b.n_atoms == 17 and b.n_mol == 3  # 17 atoms + >= 1 ghost
    assert torch.equal(b.z[:17], ref.z) and torch.equal(b.pos[:17], ref.pos) and torch.equal(b.batch[:17], ref.batch)
    assert (b.batch[17:] == 4).all() and (b.z[17:] == 1).all()
    gp = b.pos[17:]
    d = torch.cdist(gp.double(), torch.cat([ref.pos, gp]).double())
    d[:, 17:].fill_diagonal_(1e9)
    assert float(d.min()) > 5.0  # every ghost is alone within the cutoff
    assert b.y.shape == (5, 1) and b.neg_dy.shape == (24, 3)
    # weighted losses = the reference means over the real entries
    pred = torch.randn(5, 1, generator=g)
    nd = torch.randn(24, 3, generator=g)
    ly, lf = padded_losses(pred, nd, b)
    assert torch.allclose(ly, ((pred[:3] - ref.y.view(3, 1)) ** 2).mean())
    assert torch.allclose(lf, ((nd[:17] - ref.neg_dy) ** 2).mean())
    with pytest.raises(ValueError):
        pb.collate(samples * 2)  # 6 molecules > 4


def test_default_atom_buckets_cover_the_largest_batch():
    import torch
    from torchmdnet.data import Data
    from torchmdnet.module import default_atom_buckets
    ds = [Data(z=torch.ones(n, dtype=torch.long)) for n in (9, 12, 29, 17, 20) * 20]
    b = default_atom_buckets(ds, 32)
    assert b == sorted(set(b)) and b[-1] >= 29 * 32 + 1 and all(x % 32 == 0 for x in b)


def test_gradient_copy_keeps_strided_gradients():
    """training._copy_grads: contiguous gradients in one multi-tensor copy, strided ones (column blocks of
    a weight-gradient GEMM's output) one by one -- every view receives its gradient."""
    from torchmdnet.training import _copy_grads
    torch.manual_seed(0)
    flat = torch.zeros(64 + 10 + 12)
    views = [flat[:64].view(8, 8), flat[64:74], flat[74:].view(3, 4)]
    block = torch.randn(3, 5)
    grads = [torch.randn(8, 8), torch.randn(20)[::2], block[:, :4]]
    assert not grads[1].is_contiguous() and not grads[2].is_contiguous()
    _copy_grads(list(zip(views, grads)))
    for v, g in zip(views, grads):
        assert torch.equal(v, g)


def test_optimizer_steps_invalidate_the_packed_weight_cache(monkeypatch):
    """Every optimizer step of the package (training.step_reduce, LNNP.optimizer_step) drops the C++
    et_stack operator's packed-weight cache: a fused AdamW rewrites parameters without bumping the version
    counters that cache keys on."""
    from torchmdnet import _native, training
    calls = []
    monkeypatch.setattr(_native, "invalidate_stack_cache", lambda: calls.append(1))
    p = torch.nn.Parameter(torch.zeros(4))
    p.grad = torch.ones(4)
    opt = torch.optim.SGD([p], lr=0.1)
    training.step_reduce(lambda: None, opt)
    assert len(calls) == 1 and float(p[0]) == pytest.approx(-0.1)
    monkeypatch.setattr(M, "create_model", lambda args, prior=None, mean=None, std=None: TinyPotential())
    lnnp = M.LNNP(dict(lr=0.1, lr_warmup_steps=0))
    lnnp.optimizer_step(opt)
    assert len(calls) == 2
