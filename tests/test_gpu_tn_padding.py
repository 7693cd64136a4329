"""TensorNet backward kernels on a static-capacity graph (the HIP-graph training step's layout): the
per-edge gradient rows past the pair count belong to no CSR row and must come back ZERO -- the edge
and distance MLPs sum their weight gradients over all `capacity` rows (kernels.mlp_act /
kernels.linear), so stale memory there is a wrong weight gradient (found by
test_gpu_train_parity's graphed TensorNet case)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _static_graph(n_atoms, cap):
    from torchmdnet import kernels
    g = torch.Generator().manual_seed(5)
    pos = (torch.randn(n_atoms, 3, generator=g) * 1.6).cuda()
    batch = torch.zeros(n_atoms, dtype=torch.long, device="cuda")
    graph = kernels.build_graph(pos, batch, 0.0, 4.5, cap, loop=True, strategy="brute", static_capacity=cap)
    npairs = int(graph.num_pairs_dev.item())
    assert npairs < cap
    return graph, npairs


def test_tn_backward_zeroes_padding_rows():
    from torchmdnet import kernels
    N, H = 21, 64
    graph, npairs = _static_graph(N, 640)
    E = graph.n_edges
    g = torch.Generator(device="cuda").manual_seed(9)
    rn = lambda *s: torch.randn(*s, device="cuda", generator=g)  # noqa: E731
    P, Q, W, C, u = rn(N, H), rn(N, H), rn(E, 3 * H), rn(E), rn(E, 3)
    gE = rn(9, N, H)
    gP, gQ = torch.empty(N, H, device="cuda"), torch.empty(N, H, device="cuda")
    gW = torch.full((E, 3 * H), float("nan"), device="cuda")
    gC, gu = torch.full((E,), float("nan"), device="cuda"), torch.full((E, 3), float("nan"), device="cuda")
    kernels.tn_embed_bwd_launch(P, Q, W, C, u, graph, gE, gP, gQ, gW, gC, gu)
    ea, Tc, gmsg = rn(E, 3 * H), rn(9, N, H), rn(9, N, H)
    gea, gT = torch.full((E, 3 * H), float("nan"), device="cuda"), torch.empty(9, N, H, device="cuda")
    kernels.tn_message_bwd_launch(ea, Tc, graph, gmsg, gea, gT)
    torch.cuda.synchronize()
    for name, t in (("gW", gW), ("gC", gC), ("gu", gu), ("gea", gea)):
        assert torch.isfinite(t[:npairs]).all(), name
        assert (t[npairs:] == 0).all(), f"{name}: padding rows not zeroed"
