"""HIP-graph capture of the neighbour op and of the static-capacity paths (GPU).

Ports of the reference's capture tests (tests/test_neighbors.py:548-693:
test_cuda_graph_compatible_forward / _backward) plus the output contract of a captured
static-capacity build replayed with DIFFERENT pair counts (reference common.cuh:64-116: unused
capacity slots hold (-1, -1) / 0 after every call, num_pairs counts every pair found), the
captured training step fed a new batch, and its device-side guard against capacity overflow.
"""
import numpy as np
import pytest
import torch

from oracle import model_oracle as O

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _lib_loaded():
    from torchmdnet import _native
    _native.load()
    assert "libtmdnet_hip" in open("/proc/self/maps").read()  # product or debug build


def _ref_neighbors(pos, batch, loop, include_transpose, cutoff, box):
    nb, dl, d = O.neighbors(pos.detach().cpu().double().numpy(), batch.cpu().numpy(), 0.0, cutoff, loop=loop,
                            include_transpose=include_transpose,
                            box=None if box is None else box.cpu().double().numpy(), sq_compare=True)
    return O.sort_pairs(nb, dl, d)


def _grid_case(n_batches, box_type, device=DEV, dtype=torch.float32):
    """Reference test_neighbors.py:558-584 inputs."""
    torch.manual_seed(4321)
    n_per = torch.randint(3, 100, size=(n_batches,))
    batch = torch.repeat_interleave(torch.arange(n_batches, dtype=torch.int64), n_per).to(device)
    lbox = 10.0
    pos = torch.rand(int(n_per.sum()), 3, device=device, dtype=dtype) * lbox
    pos[0, :] = 0.0
    pos[1, :] = 0.0
    box = None
    if box_type is not None:
        box = torch.tensor([[lbox, 0.0, 0.0], [0.0, lbox, 0.0], [0.0, 0.0, lbox]], dtype=dtype)
    return pos, batch, box


GRID = [(s, nb, loop, tr, bt) for s in ("brute", "shared", "cell") for nb in (1, 128) for loop in (True, False)
        for tr in (True, False) for bt in (None, "triclinic", "rectangular")
        if not (bt == "triclinic" and s == "cell")]


@pytest.mark.parametrize("strategy,n_batches,loop,include_transpose,box_type", GRID)
def test_cuda_graph_compatible_forward(strategy, n_batches, loop, include_transpose, box_type):
    from torchmdnet.models.utils import OptimizedDistance
    _lib_loaded()
    cutoff = 1.0
    pos, batch, box = _grid_case(n_batches, box_type)
    pos.requires_grad_(True)
    rnb, rdl, rd = _ref_neighbors(pos, batch, loop, include_transpose, cutoff, box)
    max_num_pairs = rnb.shape[1]
    nl = OptimizedDistance(cutoff_lower=0.0, loop=loop, cutoff_upper=cutoff, max_num_pairs=max_num_pairs,
                           strategy=strategy, box=box, return_vecs=True, include_transpose=include_transpose,
                           check_errors=False, resize_to_fit=False)
    graph = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            nl(pos, batch)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    with torch.cuda.graph(graph):
        neighbors, distances, distance_vecs = nl(pos, batch)
    neighbors.fill_(0)
    graph.replay()
    torch.cuda.synchronize()
    nb, dl, d = O.sort_pairs(neighbors.cpu().numpy(), distance_vecs.detach().cpu().numpy(),
                             distances.detach().cpu().numpy())
    assert nb.shape == (2, max_num_pairs)
    assert np.array_equal(nb, rnb)
    assert np.allclose(d, rd, rtol=1e-5, atol=1e-6)
    assert np.allclose(dl, rdl, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("strategy", ["brute", "shared", "cell"])
@pytest.mark.parametrize("box_type", [None, "rectangular"])
@pytest.mark.parametrize("include_transpose", [True, False])
def test_cuda_graph_compatible_backward(strategy, box_type, include_transpose):
    """Reference test_neighbors.py:612-693: forward + distances.sum().backward() captured; the
    position gradient of the replay equals the eager one."""
    from torchmdnet.models.utils import OptimizedDistance
    _lib_loaded()
    cutoff = 1.0
    pos, batch, box = _grid_case(128, box_type)
    pos.requires_grad_(True)
    rnb, _, _ = _ref_neighbors(pos, batch, True, include_transpose, cutoff, box)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        nl = OptimizedDistance(cutoff_lower=0.0, loop=True, cutoff_upper=cutoff, max_num_pairs=rnb.shape[1],
                               strategy=strategy, box=box, return_vecs=True, include_transpose=include_transpose,
                               check_errors=False, resize_to_fit=False)
        graph = torch.cuda.CUDAGraph()
        for _ in range(3):
            _, distances, _ = nl(pos, batch)
            distances.sum().backward()
            pos.grad.data.zero_()
        torch.cuda.synchronize()
        with torch.cuda.graph(graph):
            _, distances, _ = nl(pos, batch)
            distances.sum().backward()
        pos.grad.data.zero_()
        graph.replay()
        torch.cuda.synchronize()
    torch.cuda.current_stream().wait_stream(s)
    g_graph = pos.grad.detach().clone()
    p2 = pos.detach().clone().requires_grad_(True)
    _, d2, _ = nl(p2, batch)
    (g_eager,) = torch.autograd.grad(d2.sum(), p2)
    assert torch.allclose(g_graph, g_eager, rtol=1e-5, atol=1e-5)
    assert g_graph.abs().sum() > 0


@pytest.mark.parametrize("strategy,pairs", [("brute", True), ("cell", False), ("cell", True)])
def test_static_capacity_build_replay_padding_contract(strategy, pairs):
    """One captured static-capacity build (the model's HIP-graph mode, kernels.build_graph with
    ``static_capacity``), replayed with positions that give FEWER, MORE and TOO MANY pairs than at
    capture: after every replay slots [num_pairs, cap) hold (-1, -1) / 0 (reference common.cuh:70-76),
    the transpose map -1 and the pair rows 0 there; every written index is a valid atom; the found
    pairs equal the oracle's; an overflowing replay reports num_pairs > cap and keeps every index
    in range (the list is the truncated prefix).  ``pairs``: the pair numbering (brute: inside the build;
    cell: the separate pairs.hip kernels, the large-system path's form) on the same replays."""
    from torchmdnet import kernels
    _lib_loaded()
    torch.manual_seed(11)
    n, L = 400, 16.0
    base = torch.rand(n, 3, dtype=torch.float64, device=DEV) * L
    batch = torch.repeat_interleave(torch.arange(4, device=DEV), 100)
    box = torch.eye(3, dtype=torch.float64) * L if strategy == "cell" else None
    cutoff = 3.0
    # capture at a compressed geometry (scale 0.8, more pairs), size the capacity on it; replays at
    # scale 1.0 find fewer pairs, at 0.75 / 0.6 more than the capacity (all positions stay in the box)
    pos = base * 0.8
    g0 = kernels.build_graph(pos, batch, 0.0, cutoff, 512 * n, loop=True, strategy=strategy, box=box)
    cap = int(g0.num_pairs * 1.1)
    del g0
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        kernels.build_graph(pos, batch, 0.0, cutoff, 512 * n, loop=True, strategy=strategy, box=box,
                            static_capacity=cap, pairs=pairs)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    cg = torch.cuda.CUDAGraph()
    with torch.cuda.graph(cg):
        g = kernels.build_graph(pos, batch, 0.0, cutoff, 512 * n, loop=True, strategy=strategy, box=box,
                                static_capacity=cap, pairs=pairs)
    torch.cuda.synchronize()
    seen_overflow = seen_under = False
    for scale in (0.8, 1.0, 0.75, 0.9, 0.6, 1.0, 0.8):
        pos.copy_(base * scale)
        # poison every output slot: a replay must rewrite all of them
        for t in (g.src, g.dst, g.transpose, g.row_ptr):
            t.fill_(0x7ABCDEF)
        if getattr(g, "_pairs", None) is not None:
            for t in g._pairs:
                t.fill_(0x7ABCDEF)
        g.deltas.detach().fill_(7.0)
        g.distances.detach().fill_(7.0)
        cg.replay()
        torch.cuda.synchronize()
        P = int(g.num_pairs_dev.item())
        src, dst = g.src.cpu().numpy(), g.dst.cpu().numpy()
        tr = g.transpose.cpu().numpy()
        rp = g.row_ptr.cpu().numpy()
        assert rp[0] == 0 and rp[-1] == P and np.all(np.diff(rp) >= 0)
        K = min(P, cap)
        assert np.all((src[:K] >= 0) & (src[:K] < n)) and np.all((dst[:K] >= 0) & (dst[:K] < n))
        if P <= cap:
            seen_under |= P < cap
            assert np.all(src[P:] == -1) and np.all(dst[P:] == -1) and np.all(tr[P:] == -1)
            assert torch.all(g.deltas.detach()[P:] == 0) and torch.all(g.distances.detach()[P:] == 0)
            assert np.all((tr[:P] >= 0) & (tr[:P] < P))
            assert np.array_equal(src[tr[:P]], dst[:P])
            if getattr(g, "_pairs", None) is not None:
                pr = g._pairs[0].cpu().numpy()
                assert np.all(pr[P:] == 0) and np.all((pr[:P] >= 0) & (pr[:P] < (P + n) // 2))
            ref, _, _ = O.neighbors(pos.cpu().numpy(), batch.cpu().numpy(), 0.0, cutoff, loop=True,
                                    box=None if box is None else box.numpy(), sq_compare=True)
            mine = np.stack([src[:P], dst[:P]]).astype(np.int64)
            assert np.array_equal(mine[:, np.lexsort(mine)], ref[:, np.lexsort(ref)])
        else:
            seen_overflow = True
            assert bool(g.overflow.item())
            assert np.all((tr[:K] >= -1) & (tr[:K] < cap))
        if getattr(g, "_pairs", None) is not None:
            # every pair row index and every pair's canonical edge stays in range, also when the list
            # overflowed (consumers gather r / f through pair_edge: an unwritten slot would be a wild index)
            pr, pe = g._pairs[0].cpu().numpy(), g._pairs[1].cpu().numpy()
            assert np.all((pr >= 0) & (pr < pe.shape[0])) and np.all((pe >= 0) & (pe < cap))
            if P <= cap:
                canon = src[:P] >= dst[:P]
                assert np.array_equal(pe[pr[:P][canon]], np.nonzero(canon)[0])
    assert seen_overflow and seen_under


def _small_et(precision=64, **kw):
    from conftest import yaml_args
    from torchmdnet.models.model import create_model
    torch.manual_seed(1234)
    args = yaml_args("equivariant-transformer", embedding_dimension=32, num_layers=2, num_rbf=16, num_heads=4,
                     derivative=True, output_model="Scalar", precision=precision, **kw)
    return create_model(args).to(DEV)


def test_graphed_train_step_takes_new_species_and_batch():
    """GraphedTrainStep.step copies z and batch too: a new batch of the same layout
    gives the eager LNNPStep's loss and gradients."""
    from torchmdnet.training import GraphedTrainStep, LNNPStep
    m = _small_et()
    z, pos, batch = O.qm9_like(4)
    z, pos, batch = z.to(DEV), pos.to(DEV), batch.to(DEV)
    y = torch.randn(4, 1, dtype=torch.float64, device=DEV)
    f = torch.randn(pos.shape, dtype=torch.float64, device=DEV)
    gtr = GraphedTrainStep(m, z, pos, batch, y, f, lr=0.0)
    z2 = z.clone()
    z2[z2 == 1] = 6
    z2[z2 == 8] = 1
    b2 = batch.clone()
    first3 = int((batch == 3).nonzero()[0])
    b2[first3] = 2  # the first atom of the last molecule joins the third: 4 molecules, new grouping
    y2 = torch.randn(4, 1, dtype=torch.float64, device=DEV)
    y2[3] = 0.0
    loss_g = gtr.step(z=z2, pos=pos + 0.01, batch=b2, y=y2).clone()
    g_graph = [p.grad.clone() for p in m.parameters()]
    gtr.check_capacity()
    gtr.release()
    with pytest.raises(ValueError):
        gtr.step(z=z2[:-1])
    ref = LNNPStep(m, lr=0.0)
    ref.opt.zero_grad(set_to_none=True)
    loss_r = ref.loss(z2, pos + 0.01, b2, y2, f)
    ref.backward(loss_r)
    assert torch.allclose(loss_g, loss_r.detach(), rtol=1e-10)
    for a, b in zip(g_graph, [p.grad for p in m.parameters()]):
        assert torch.allclose(a, b, rtol=1e-9, atol=1e-11)


def test_graphed_train_step_skips_overflowing_step():
    """a replay whose pair count exceeds the captured capacity must not reach the
    weights.  The skip flag rides in the gradient buffer and AdamW's found_inf skips the update on
    the device; check_capacity raises afterwards."""
    from torchmdnet.training import GraphedTrainStep
    m = _small_et(cutoff_upper=2.0)  # a short cutoff, so compressing the molecules adds pairs
    z, pos, batch = O.qm9_like(4)
    z, pos, batch = z.to(DEV), pos.to(DEV), batch.to(DEV)
    y = torch.randn(4, 1, dtype=torch.float64, device=DEV)
    f = torch.randn(pos.shape, dtype=torch.float64, device=DEV)
    gtr = GraphedTrainStep(m, z, pos, batch, y, f, lr=1e-2)
    gtr.step()
    gtr.check_capacity()
    before = [p.detach().clone() for p in m.parameters()]
    gtr.step(pos=pos * 0.3)  # compressed molecules: far more pairs than the capacity
    assert gtr.skipped_steps == 1
    for a, p in zip(before, m.parameters()):
        assert torch.equal(a, p.detach())
    with pytest.raises(RuntimeError, match="capacity"):
        gtr.check_capacity()
    gtr.step(pos=pos)  # back in range: updates again
    assert any(not torch.equal(a, p.detach()) for a, p in zip(before, m.parameters()))
    gtr.release()


@pytest.mark.parametrize("fused", [True, False])
def test_graph_capture_of_the_large_system_path(fused, monkeypatch):
    """the renumbered large-system path (Morton renumbering, cell list in a periodic box,
    planar rows, and -- fused -- the fused-projection kernels, or the pair-row path with the merged dr
    backward) captured in one HIP graph: replays on fresh coordinates equal eager evaluations."""
    from conftest import yaml_args
    from torchmdnet import et_stack, kernels
    from torchmdnet.graphs import GraphedEnergyForces
    from torchmdnet.models.model import create_model
    monkeypatch.setattr(kernels, "REORDER_MIN_ATOMS", 0)
    monkeypatch.setattr(et_stack, "PLANAR_MIN_EDGES", 0)
    if fused:
        monkeypatch.setattr(et_stack, "FEP_MIN_EDGES", 0)
    else:
        monkeypatch.setattr(et_stack, "FEP", "0")
    prev = kernels.set_tuning(kernels.TUNE_ET_MERGED_MIN_NODES, 0)
    try:
        torch.manual_seed(0)
        m = create_model(yaml_args("equivariant-transformer", embedding_dimension=128, num_layers=3, num_rbf=64,
                                   num_heads=8, max_num_neighbors=128, derivative=True)).to(DEV)
        n = 3000
        g = torch.Generator().manual_seed(5)
        L = (n / 0.1003) ** (1.0 / 3.0)
        pos = (torch.rand(n, 3, generator=g, dtype=torch.float64) * L).float().to(DEV)
        z = torch.tensor([8, 1, 1], dtype=torch.long).repeat(n // 3 + 1)[:n].to(DEV)
        batch = torch.zeros(n, dtype=torch.long, device=DEV)
        d = m.representation_model.distance
        d.box = torch.eye(3, dtype=torch.float32) * L
        d.use_periodic = True
        d.strategy = "cell"
        gm = GraphedEnergyForces(m, z, pos, batch)
        for step in range(3):
            p = pos + 0.05 * torch.randn(pos.shape, generator=torch.Generator().manual_seed(step)).to(DEV)
            y, f = gm(p)
            y, f = y.clone(), f.clone()
            ye, fe = m(z, p.clone(), batch)
            assert float((y - ye).abs().max() / ye.abs().max()) < 1e-5
            assert float((f - fe).abs().max() / fe.abs().max()) < 1e-5
        gm.check_capacity()
        gm.release()
    finally:
        kernels.set_tuning(kernels.TUNE_ET_MERGED_MIN_NODES, prev)
