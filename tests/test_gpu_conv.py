"""GPU parity of the sv2n GATConv (C-ABI kernels) against the PyG-2.3.0
restatement in oracle/ on identical inputs and weights; tolerance in
tests/helpers.py (1e-5, scaled by max(1, |ref|))."""
import pytest
import torch

from helpers import assert_parity, block_graphs, dense_keep_to_edges, float64_twin, twin_conv

pytestmark = pytest.mark.gpu


def _run(mine, ref, x, ei, ea, dev):
    ref64 = float64_twin(ref)
    mine = mine.to(dev)
    xg = x.clone().to(dev).requires_grad_(True)
    xr = x.clone().requires_grad_(True)
    x64 = x.clone().double().requires_grad_(True)
    out = mine(xg, ei.to(dev), ea.to(dev) if ea is not None else None)
    rout = ref(xr, ei, ea)
    r64 = ref64(x64, ei, ea.double() if ea is not None else None)
    w = torch.randn_like(rout)
    (out * w.to(dev)).sum().backward()
    (rout * w).sum().backward()
    (r64 * w.double()).sum().backward()
    assert_parity(out, rout, r64, what="forward")
    assert_parity(xg.grad, xr.grad, x64.grad, what="dx")
    for (name, p), (_, q), (_, q64) in zip(mine.named_parameters(), ref.named_parameters(),
                                           ref64.named_parameters()):
        assert_parity(p.grad, q.grad, q64.grad, what=f"d{name}")
    return out


@pytest.mark.parametrize("concat", [True, False])
@pytest.mark.parametrize("heads,C", [(1, 5), (4, 8), (6, 3)])
def test_canonical(dev, concat, heads, C):
    B, n, S = 3, 30, 2
    mine, ref = twin_conv(n * S, C, heads, concat, 3 * S, seed=heads)
    torch.manual_seed(1)
    x = torch.randn(B * n, n * S)
    ei = block_graphs(B, n)
    ea = torch.randn(ei.size(1), 3 * S)
    _run(mine, ref, x, ei, ea, dev)


def test_no_edge_attr(dev):
    """edge_attr=None (the GNNExplainer call, 6_results.ipynb:1284-1287)."""
    mine, ref = twin_conv(12, 7, 4, True, 6, seed=3)
    x = torch.randn(2 * 30, 12)
    _run(mine, ref, x, block_graphs(2, 30), None, dev)


def test_no_edge_dim(dev):
    mine, ref = twin_conv(12, 7, 2, False, None, seed=4)
    x = torch.randn(2 * 30, 12)
    _run(mine, ref, x, block_graphs(2, 30), torch.randn(2 * 870, 6), dev)


def test_one_dim_edge_attr(dev):
    """1-D edge_attr viewed as [E, 1] (PyG edge_update; CovarianceSparseDataset)."""
    mine, ref = twin_conv(10, 4, 3, True, 1, seed=5)
    ei = block_graphs(2, 30)
    _run(mine, ref, torch.randn(60, 10), ei, torch.randn(ei.size(1)), dev)


@pytest.mark.parametrize("keep_frac,shuffle,loops", [(1.0, True, False), (0.6, True, False),
                                                     (0.3, False, True), (1.0, False, True)])
def test_block_layouts(dev, keep_frac, shuffle, loops):
    """Non-canonical edge order, missing edges (incl. nodes with no in-edges),
    and self loops in the input (PyG removes them before adding its own)."""
    B, n = 4, 30
    mine, ref = twin_conv(9, 6, 4, True, 5, seed=6)
    ei = block_graphs(B, n, keep_frac, shuffle, loops, seed=11)
    if keep_frac < 0.5:  # isolate node 5 of graph 1 completely
        ei = ei[:, ei[1] != n + 5]
    _run(mine, ref, torch.randn(B * n, 9), ei, torch.randn(ei.size(1), 5), dev)


@pytest.mark.parametrize("n", [1, 2, 5, 17, 32])
def test_graph_sizes(dev, n):
    B = 3
    mine, ref = twin_conv(8, 4, 2, True, 3, seed=n)
    ei = block_graphs(B, n)
    _run(mine, ref, torch.randn(B * n, 8), ei, torch.randn(ei.size(1), 3), dev)


@pytest.mark.parametrize("n,heads", [(3, 1), (7, 3), (31, 1), (30, 3)])
def test_edge_order_partial_slots(dev, n, heads):
    """Canonical batches carry the edge logits in edge order [B*n(n-1)][H]:
    with H odd a graph's block is neither a multiple of four floats nor
    16-B aligned (the attention kernels' clamped scalar path)."""
    B = 5
    mine, ref = twin_conv(6, 4, heads, True, 3, seed=n + heads)
    ei = block_graphs(B, n)
    _run(mine, ref, torch.randn(B * n, 6), ei, torch.randn(ei.size(1), 3), dev)


@pytest.mark.parametrize("slope", [0.05, 0.8])
def test_negative_slope(dev, slope):
    mine, ref = twin_conv(12, 6, 3, False, 4, slope=slope, seed=8)
    ei = block_graphs(2, 30)
    _run(mine, ref, torch.randn(60, 12) * 3, ei, torch.randn(ei.size(1), 4), dev)


def test_attention_dropout(dev):
    """dropout_att: the kernel applies a [B,H,n,n] keep mask drawn by torch; the
    oracle is fed the same mask in PyG edge order."""
    B, n, H, p = 2, 30, 4, 0.3
    mine, ref = twin_conv(10, 5, H, True, 3, dropout=p, seed=9)
    mine.train()
    ref.train()
    ei = block_graphs(B, n)
    torch.cuda.manual_seed(123)
    keep = (torch.rand(B, H, 32, 32, device=dev) >= p).to(torch.uint8).cpu()[:, :, :n, :n]
    ref.attn_keep = dense_keep_to_edges(keep, ei, n)
    torch.cuda.manual_seed(123)
    _run(mine, ref, torch.randn(B * n, 10), ei, torch.randn(ei.size(1), 3), dev)


def test_deterministic(dev):
    mine, _ = twin_conv(40, 16, 4, True, 6, seed=10)
    mine = mine.to(dev)
    x = torch.randn(64 * 30, 40, device=dev)
    ei = block_graphs(64, 30).to(dev)
    ea = torch.randn(ei.size(1), 6, device=dev)
    a = mine(x, ei, ea)
    b = mine(x, ei, ea)
    assert torch.equal(a, b)


def test_cpu_tensors_fail_loudly():
    from spotv2net_amd import GATConv
    conv = GATConv(4, 2, heads=1, edge_dim=1)
    ei = block_graphs(1, 3)
    with pytest.raises((RuntimeError, NotImplementedError)):
        conv(torch.randn(3, 4), ei, torch.randn(ei.size(1), 1))


@pytest.mark.parametrize("concat", [True, False])
def test_no_bias(dev, concat):
    """GATConv(bias=False): the attention kernels take a NULL bias."""
    mine, ref = twin_conv(12, 7, 3, concat, 4, seed=12, bias=False)
    ei = block_graphs(2, 30)
    _run(mine, ref, torch.randn(60, 12), ei, torch.randn(ei.size(1), 4), dev)


@pytest.mark.parametrize("B,heads,C,concat", [
    (3, 6, 70, True),     # fwd 4 splits; bwd 6 splits of 1 head, 3 chunks over 2 waves
    (3, 6, 70, False),    # the same for the head mean (bias partial from head 0's split)
    (3, 2, 260, False),   # fwd: 9 tiles over 2 splits (mean over heads per tile); bwd 4 waves
    (3, 2, 100, True),    # bwd: 2 splits, a head's 4 chunks over 4 waves
    (300, 3, 40, True),   # bwd: 2 splits of 2 + 1 heads (the last split half empty)
    (100, 5, 40, False),  # bwd: 5 splits of 1 head, 2 chunks over 2 waves
    (1024, 8, 4, True),   # 8 heads with the batch filling the chip: bwd 2 splits of 4 heads
                          # (at B = 1000 / 1100 these seeds put an attention logit on the
                          # leaky-ReLU kink)
])
def test_workgroup_splits(dev, B, heads, C, concat):
    """n <= 32 attention with a graph's work spread over several workgroups
    (sv2n_attn_canon.hip: canon_fwd_splits / canon_bwd_plan pick the split
    from the batch size; C3's 128 graphs of 6 x 500 columns run 4 forward and
    6 backward workgroups per graph)."""
    n = 30
    mine, ref = twin_conv(12, C, heads, concat, 3, seed=B + heads)
    torch.manual_seed(B)
    x = torch.randn(B * n, 12)
    ei = block_graphs(B, n)
    _run(mine, ref, x, ei, torch.randn(ei.size(1), 3), dev)
