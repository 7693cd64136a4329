"""Generate golden fixtures by running the REFERENCE implementation (raimis/torchmd-net, read-only at
/root/reference) on CPU in this container.

Recipe: ``oracle/pyref/setup_ref.sh`` copies the reference package to /tmp/tmdref (outside the
repo), builds its CPU neighbour op there and adds the test shims for PyG / torch_scatter.  This script
must run in a process whose ``sys.path`` holds only that copy (``run_reference_fixtures.sh`` does it),
so that ``import torchmdnet`` is the reference, not this repo's package.

Only numeric data (inputs, expected outputs, per-parameter checksums, small state dicts) is written,
as ``.npz`` files under tests/golden/.  No reference source or bytecode enters the repo.
"""
import os
import sys
import random

import numpy as np
import torch

OUT = os.path.dirname(os.path.abspath(__file__))
EXAMPLES = "/root/reference/examples"

import yaml  # noqa: E402
from torchmdnet.models.model import create_model  # noqa: E402  (the reference)
import torchmdnet.models.utils as ref_utils  # noqa: E402
import torchmdnet.models.tensornet as ref_tn  # noqa: E402


def seed_everything(s):
    random.seed(s)
    np.random.seed(s)
    torch.manual_seed(s)


def base_args(model, **kw):
    cfg = "TensorNet-QM9.yaml" if model == "tensornet" else "ET-QM9.yaml"
    with open(os.path.join(EXAMPLES, cfg)) as f:
        args = yaml.load(f, Loader=yaml.SafeLoader)
    args.setdefault("precision", 32)
    args["model"] = model
    args["prior_model"] = None
    args.update(kw)
    return args


def qm9_like(n_mol, gen_seed=1):
    """SURVEY.md §8(d) QM9-like generator (the exact tensors are stored in each fixture)."""
    g = torch.Generator().manual_seed(gen_seed)
    zs, ps, bs = [], [], []
    for m in range(n_mol):
        n = int(torch.randint(9, 30, (1,), generator=g))
        heavy = n // 2
        z = torch.ones(n, dtype=torch.long)
        z[:heavy] = torch.tensor([6, 7, 8, 9])[torch.randint(0, 4, (heavy,), generator=g)]
        zs.append(z)
        ps.append(torch.randn(n, 3, generator=g, dtype=torch.float64) * 1.6)
        bs.append(torch.full((n,), m, dtype=torch.long))
    return torch.cat(zs), torch.cat(ps), torch.cat(bs)


def aspirin_like(n_mol, gen_seed=2):
    g = torch.Generator().manual_seed(gen_seed)
    z1 = torch.tensor([6] * 9 + [1] * 8 + [8] * 4, dtype=torch.long)
    z = z1.repeat(n_mol)
    pos = torch.randn(len(z), 3, generator=g, dtype=torch.float64) * 1.6
    batch = torch.arange(n_mol).repeat_interleave(len(z1))
    return z, pos, batch


def param_checksums(model):
    out = {}
    for name, p in model.state_dict().items():
        a = p.detach().double()
        out["ck/" + name] = np.array([a.sum().item(), (a * a).sum().item(), a.numel()], dtype=np.float64)
    return out


def state_dict_arrays(model):
    return {"sd/" + k: v.detach().cpu().numpy() for k, v in model.state_dict().items()}


def run_model(model, z, pos, batch, dtype, second_order=True):
    pos = pos.to(dtype).clone()
    y, neg_dy = model(z, pos, batch)
    res = {"z": z.numpy(), "pos": pos.detach().numpy(), "batch": batch.numpy(),
           "y": y.detach().numpy(), "neg_dy": neg_dy.detach().numpy()}
    if second_order:
        # force-loss double backward: the LNNP training objective shape (module.py:165-177)
        loss = (y ** 2).sum() + (neg_dy ** 2).sum()
        params = [p for p in model.parameters() if p.requires_grad]
        names = [n for n, p in model.named_parameters() if p.requires_grad]
        grads = torch.autograd.grad(loss, params, allow_unused=True)
        for n, gr in zip(names, grads):
            res["g2/" + n] = (np.zeros(1) if gr is None else gr.detach().numpy())
    return res


def capture_layers(model, store):
    rep = model.representation_model
    if hasattr(rep, "attention_layers"):
        for li, layer in enumerate(rep.attention_layers):
            def hook(mod, inp, out, li=li):
                store[f"layer{li}/dx"] = out[0].detach().numpy().copy()
                store[f"layer{li}/dvec"] = out[1].detach().numpy().copy()
            layer.register_forward_hook(hook)

    def rhook(mod, inp, out):
        store["rep/x"] = out[0].detach().numpy().copy()
        if out[1] is not None:
            store["rep/vec"] = out[1].detach().numpy().copy()
    rep.register_forward_hook(rhook)


def save(name, d):
    path = os.path.join(OUT, name)
    np.savez_compressed(path, **d)
    print("wrote", path, os.path.getsize(path), "bytes")


# --------------------------------------------------------------------------- neighbour lists
def sort_nl(nb, dv, d):
    order = np.lexsort(nb)
    return nb[:, order], dv[order], d[order]


def gen_neighbors():
    kern = ref_utils.get_neighbor_pairs_kernel
    d = {}
    cases = []
    torch.manual_seed(4321)
    for n_batches in (1, 3, 16):
        for box_type in (None, "rectangular", "triclinic"):
            for dtype in (torch.float32, torch.float64):
                if n_batches == 16 and dtype == torch.float64:
                    continue
                n_per = torch.randint(3, 100, (n_batches,))
                batch = torch.repeat_interleave(torch.arange(n_batches), n_per)
                lbox = 10.0
                pos = torch.rand(int(n_per.sum()), 3, dtype=dtype) * lbox - 10.0 * lbox
                pos[0] = 0.0
                pos[1] = 0.0
                if box_type is None:
                    box = torch.empty((0, 0), dtype=dtype)
                elif box_type == "rectangular":
                    box = torch.tensor([[lbox, 0, 0], [0, lbox, 0], [0, 0, lbox]], dtype=dtype)
                else:
                    box = torch.tensor([[lbox, 0, 0], [0.1, lbox, 0], [0.3, 0.2, lbox]], dtype=dtype)
                for cutoff in ((1.0,) if n_batches == 16 else (1.0, 4.9)):
                    for loop in (False, True):
                        for tr in (False, True):
                            k = len(cases)
                            nb, dv, dist, npairs = kern("brute", pos, batch, box, box_type is not None,
                                                        0.0, cutoff, 10 ** 7, loop, tr)
                            nb, dv, dist = sort_nl(nb.numpy(), dv.numpy(), dist.numpy())
                            d[f"c{k}/pos"] = pos.numpy()
                            d[f"c{k}/batch"] = batch.numpy()
                            d[f"c{k}/box"] = box.numpy()
                            d[f"c{k}/params"] = np.array([cutoff, loop, tr, box_type is not None], dtype=np.float64)
                            d[f"c{k}/neighbors"] = nb.astype(np.int32)
                            d[f"c{k}/deltas"] = dv
                            d[f"c{k}/distances"] = dist
                            d[f"c{k}/num_pairs"] = np.array([int(npairs[0])])
                            cases.append(k)
    d["ncases"] = np.array([len(cases)])
    save("neighbors_ref.npz", d)


# --------------------------------------------------------------------------- ET
def gen_et():
    for dtype, tag in ((torch.float64, "f64"), (torch.float32, "f32")):
        prec = 64 if dtype == torch.float64 else 32
        args = base_args("equivariant-transformer", embedding_dimension=32, num_layers=2, num_rbf=16,
                         num_heads=4, max_num_neighbors=32, derivative=True, output_model="Scalar",
                         precision=prec)
        seed_everything(1234)
        model = create_model(args)
        z, pos, batch = qm9_like(3)
        store = {}
        capture_layers(model, store)
        res = run_model(model, z, pos, batch, dtype)
        res.update(store)
        res.update(state_dict_arrays(model))
        save(f"et_tiny_{tag}.npz", res)

    # C2 (ET-QM9 at 128 channels): seed-reproduced weights (checksums only) + outputs, f32 and f64
    for dtype, tag in ((torch.float32, "f32"), (torch.float64, "f64")):
        prec = 64 if dtype == torch.float64 else 32
        args = base_args("equivariant-transformer", embedding_dimension=128, derivative=True,
                         output_model="Scalar", precision=prec)
        seed_everything(1234)
        model = create_model(args)
        res = param_checksums(model)
        z, pos, batch = qm9_like(4)
        res.update(run_model(model, z, pos, batch, dtype, second_order=False))
        save(f"et_c2_{tag}.npz", res)


# --------------------------------------------------------------------------- TensorNet
def padded_kernel(orig):
    """Emulates the CUDA op's output contract on the CPU op (common.cuh:70-76): outputs padded to
    max_num_pairs with (-1,-1) neighbours and zero deltas/distances."""
    def k(strategy, positions, batch, box_vectors, use_periodic, cutoff_lower, cutoff_upper,
          max_num_pairs, loop, include_transpose):
        nb, dv, d, n = orig(strategy, positions, batch, box_vectors, use_periodic, cutoff_lower,
                            cutoff_upper, max_num_pairs, loop, include_transpose)
        cap = int(max_num_pairs)
        p = nb.shape[1]
        if p > cap:
            raise RuntimeError("fixture case overflowed capacity")
        nbp = torch.full((2, cap), -1, dtype=nb.dtype)
        nbp[:, :p] = nb
        dvp = torch.zeros((cap, 3), dtype=dv.dtype)
        dvp[:p] = dv
        dp = torch.zeros((cap,), dtype=d.dtype)
        dp[:p] = d
        return nbp, dvp, dp, n
    return k


def gen_tensornet():
    orig = ref_utils.get_neighbor_pairs_kernel
    for static in (True, False):
        for group in ("O(3)", "SO(3)"):
            for dtype, tag in ((torch.float64, "f64"), (torch.float32, "f32")):
                if dtype == torch.float32 and not (static and group == "O(3)"):
                    continue
                prec = 64 if dtype == torch.float64 else 32
                ref_utils.get_neighbor_pairs_kernel = padded_kernel(orig) if static else orig
                import torchmdnet.models.utils as u
                u.get_neighbor_pairs_kernel = ref_utils.get_neighbor_pairs_kernel
                args = base_args("tensornet", embedding_dimension=32, num_layers=2, num_rbf=16,
                                 max_num_neighbors=32, cutoff_upper=4.5, derivative=True,
                                 output_model="Scalar", precision=prec,
                                 equivariance_invariance_group=group)
                seed_everything(1234)
                model = create_model(args)
                model.representation_model.static_shapes = static
                model.representation_model.distance.resize_to_fit = not static
                z, pos, batch = aspirin_like(2)
                store = {}
                capture_layers(model, store)
                res = run_model(model, z, pos, batch, dtype)
                res.update(store)
                res.update(state_dict_arrays(model))
                g = "o3" if group == "O(3)" else "so3"
                save(f"tn_tiny_{g}_{'static' if static else 'dyn'}_{tag}.npz", res)
    # C3 (TensorNet-rMD17: 128 ch, 2 layers, 32 rbf, cutoff 4.5, max_nbr 32), padded (CUDA) semantics
    ref_utils.get_neighbor_pairs_kernel = padded_kernel(orig)
    with open(os.path.join(EXAMPLES, "TensorNet-rMD17.yaml")) as f:
        args = yaml.load(f, Loader=yaml.SafeLoader)
    args["prior_model"] = None
    args["precision"] = 32
    seed_everything(1234)
    model = create_model(args)
    res = param_checksums(model)
    z, pos, batch = aspirin_like(2)
    res.update(run_model(model, z, pos, batch, torch.float32, second_order=False))
    save("tn_c3_f32.npz", res)
    ref_utils.get_neighbor_pairs_kernel = orig


# --------------------------------------------------------------------------- seed reproduction
def gen_seed_checksums():
    """Parameter checksums of create_model(ET-QM9.yaml / TensorNet-QM9.yaml) after seed 1234 and the
    example batch that tests/test_model.py:143-189 feeds them (expected.pkl pins the outputs)."""
    res = {}
    for model_name, tag in (("equivariant-transformer", "et"), ("tensornet", "tn")):
        seed_everything(1234)
        args = base_args(model_name, derivative=True, output_model="Scalar")
        model = create_model(args)
        for k, v in param_checksums(model).items():
            res[f"{tag}/{k}"] = v
        zs = torch.tensor([1, 6, 7, 8, 9], dtype=torch.long)
        z = zs[torch.randint(0, len(zs), (5,))]
        pos = torch.randn(len(z), 3)
        batch = torch.zeros(len(z), dtype=torch.long)
        batch[len(batch) // 2:] = 1
        y, neg_dy = model(z, pos, batch)
        res[f"{tag}/z"] = z.numpy()
        res[f"{tag}/pos"] = pos.detach().numpy()
        res[f"{tag}/batch"] = batch.numpy()
        res[f"{tag}/y"] = y.detach().numpy()
        res[f"{tag}/neg_dy"] = neg_dy.detach().numpy()
    save("seed1234_qm9.npz", res)


# --------------------------------------------------------------------------- edge cases (round 2)
def gen_edge_cases():
    """ET with a lower cutoff (shifted CosineCutoff, neighbour lower bound; reference
    models/utils.py:362-390, neighbors_cpu.cpp:82-86) and ET with the Atomref prior of ET-QM9.yaml
    (priors/atomref.py:8-42) with non-zero per-element references."""
    for name, extra in (("et_tiny_cl2_f64.npz", dict(cutoff_lower=2.0, cutoff_upper=5.0)),
                        ("et_tiny_atomref_f64.npz", dict(prior_model="Atomref", prior_args={"max_z": 100}))):
        args = base_args("equivariant-transformer", embedding_dimension=32, num_layers=2, num_rbf=16,
                         num_heads=4, max_num_neighbors=32, derivative=True, output_model="Scalar",
                         precision=64)
        args.update(extra)
        seed_everything(1234)
        model = create_model(args)
        if "prior_model" in extra:
            g = torch.Generator().manual_seed(77)
            w = model.prior_model[0].atomref.weight
            w.data.copy_(torch.randn(w.shape, generator=g, dtype=w.dtype))
        z, pos, batch = qm9_like(3)
        res = run_model(model, z, pos, batch, torch.float64)
        res.update(state_dict_arrays(model))
        save(name, res)


# --------------------------------------------------------------------------- activations (round 3)
def gen_activations():
    """ET with non-SiLU `activation` / `attn_activation` (reference act_class_mapping,
    models/utils.py:579-584; EquivariantMultiHeadAttention, torchmd_et.py:208-347): energies, forces and
    the force-loss parameter gradients."""
    for name, act, attn in (("et_tiny_act_tanh_ssp_f64.npz", "tanh", "ssp"),
                            ("et_tiny_act_sigmoid_tanh_f64.npz", "sigmoid", "tanh")):
        args = base_args("equivariant-transformer", embedding_dimension=32, num_layers=2, num_rbf=16,
                         num_heads=4, max_num_neighbors=32, derivative=True, output_model="Scalar",
                         precision=64, activation=act, attn_activation=attn)
        seed_everything(1234)
        model = create_model(args)
        z, pos, batch = qm9_like(3)
        res = run_model(model, z, pos, batch, torch.float64)
        res.update(state_dict_arrays(model))
        save(name, res)


def gen_splits():
    """utils.make_splits / train_val_test_split index sets (reference torchmdnet/utils.py:54-139)."""
    from torchmdnet.utils import make_splits
    res = {}
    cases = [(1000, 0.8, 0.1, None, 1), (100, 50, 20, 30, 2), (200, 0.5, 0.25, 0.25, 3),
             (131, 0.7, 0.2, 0.1, 4), (57, None, 10, 0.2, 5), (1000, 800, None, 0.1, 12345)]
    for k, (n, tr, va, te, seed) in enumerate(cases):
        a, b, c = make_splits(n, tr, va, te, seed)
        res[f"s{k}/args"] = np.array([n, -1 if tr is None else tr, -1 if va is None else va,
                                      -1 if te is None else te, seed], dtype=np.float64)
        res[f"s{k}/is_float"] = np.array([isinstance(x, float) for x in (tr, va, te)])
        res[f"s{k}/train"], res[f"s{k}/val"], res[f"s{k}/test"] = a.numpy(), b.numpy(), c.numpy()
    order = np.random.default_rng(9).permutation(50)
    a, b, c = make_splits(50, 30, 10, 10, 0, order=order)
    res["order/order"] = order
    res["order/train"], res["order/val"], res["order/test"] = a.numpy(), b.numpy(), c.numpy()
    res["ncases"] = np.array([len(cases)])
    save("splits_ref.npz", res)

# --------------------------------------------------------------------------- periodic models (round 5)
def water_box(n, gen_seed=11):
    """SURVEY.md §8(d) water box at small n: z = (O, H, H) repeated, uniform positions in a cube of
    the water number density 0.1003 / A^3 (the exact tensors are stored in each fixture)."""
    g = torch.Generator().manual_seed(gen_seed)
    L = (n / 0.1003) ** (1.0 / 3.0)
    z = torch.tensor([8, 1, 1], dtype=torch.long).repeat(n // 3 + 1)[:n]
    pos = torch.rand(n, 3, generator=g, dtype=torch.float64) * L
    return z, pos, torch.zeros(n, dtype=torch.long), L


def gen_periodic():
    """ET-tiny and TensorNet-tiny (static padded and dynamic shapes) on a rectangular periodic box: the
    reference CPU neighbour op's minimum image (neighbors_cpu.cpp:63-70) through the whole model,
    energies, forces and the force-loss parameter gradients."""
    orig = ref_utils.get_neighbor_pairs_kernel
    n = 120
    z, pos, batch, L = water_box(n)
    box = torch.eye(3, dtype=torch.float64) * L

    def set_box(model, dtype):
        d = model.representation_model.distance
        d.box = box.to(dtype)
        d.use_periodic = True

    args = base_args("equivariant-transformer", embedding_dimension=32, num_layers=2, num_rbf=16, num_heads=4,
                     max_num_neighbors=64, derivative=True, output_model="Scalar", precision=64)
    seed_everything(1234)
    model = create_model(args)
    set_box(model, torch.float64)
    res = run_model(model, z, pos, batch, torch.float64)
    res.update(state_dict_arrays(model))
    res["box"] = box.numpy()
    save("et_tiny_periodic_f64.npz", res)
    for static in (True, False):
        ref_utils.get_neighbor_pairs_kernel = padded_kernel(orig) if static else orig
        import torchmdnet.models.utils as u
        u.get_neighbor_pairs_kernel = ref_utils.get_neighbor_pairs_kernel
        args = base_args("tensornet", embedding_dimension=32, num_layers=2, num_rbf=16, max_num_neighbors=64,
                         cutoff_upper=4.5, derivative=True, output_model="Scalar", precision=64)
        seed_everything(1234)
        model = create_model(args)
        model.representation_model.static_shapes = static
        model.representation_model.distance.resize_to_fit = not static
        set_box(model, torch.float64)
        res = run_model(model, z, pos, batch, torch.float64)
        res.update(state_dict_arrays(model))
        res["box"] = box.numpy()
        save(f"tn_tiny_periodic_{'static' if static else 'dyn'}_f64.npz", res)
    ref_utils.get_neighbor_pairs_kernel = orig
    import torchmdnet.models.utils as u
    u.get_neighbor_pairs_kernel = orig


if __name__ == "__main__":
    which = sys.argv[1:] or ["neighbors", "et", "tensornet", "seed", "edge", "splits", "acts", "periodic"]
    if "periodic" in which:
        gen_periodic()
    if "acts" in which:
        gen_activations()
    if "edge" in which:
        gen_edge_cases()
    if "splits" in which:
        gen_splits()
    if "neighbors" in which:
        gen_neighbors()
    if "et" in which:
        gen_et()
    if "tensornet" in which:
        gen_tensornet()
    if "seed" in which:
        gen_seed_checksums()
