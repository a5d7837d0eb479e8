"""GPU parity of the target-row-tiled attention path (32 < n <= 256 nodes per
graph: the C5 stress shapes of SURVEY.md §8d) against the PyG-2.3.0
restatement, same tolerance rule as test_gpu_conv (helpers.assert_parity)."""
import pytest
import torch

from helpers import (assert_parity, block_graphs, dense_keep_to_edges, float64_twin, twin_conv,
                     twin_model)
from test_gpu_conv import _run

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [33, 64, 100, 256])
@pytest.mark.parametrize("concat", [True, False])
def test_tiled_canonical(dev, n, concat):
    B, H, C = 2, 4, 16
    mine, ref = twin_conv(24, C, H, concat, 6, seed=n)
    torch.manual_seed(2)
    ei = block_graphs(B, n)
    _run(mine, ref, torch.randn(B * n, 24), ei, torch.randn(ei.size(1), 6), dev)


@pytest.mark.parametrize("heads,C", [(1, 5), (8, 16), (3, 33), (2, 64)])
def test_tiled_channel_widths(dev, heads, C):
    B, n = 2, 48
    mine, ref = twin_conv(20, C, heads, True, 3, seed=C)
    ei = block_graphs(B, n)
    _run(mine, ref, torch.randn(B * n, 20), ei, torch.randn(ei.size(1), 3), dev)


@pytest.mark.parametrize("n,keep_frac,shuffle,loops", [(64, 1.0, True, False),
                                                       (100, 0.5, True, True),
                                                       (256, 0.2, False, True),
                                                       (40, 0.05, True, False)])
def test_tiled_block_layouts(dev, n, keep_frac, shuffle, loops):
    """Arbitrary edge order, missing edges (multi-word row masks, isolated
    targets) and input self loops on the tiled path."""
    B = 2
    mine, ref = twin_conv(10, 8, 4, True, 5, seed=7)
    ei = block_graphs(B, n, keep_frac, shuffle, loops, seed=n)
    ei = ei[:, ei[1] != n + 3]  # target 3 of graph 1 has no in-edges
    _run(mine, ref, torch.randn(B * n, 10), ei, torch.randn(ei.size(1), 5), dev)


def test_tiled_no_edge_attr(dev):
    mine, ref = twin_conv(12, 7, 4, False, 6, seed=3)
    _run(mine, ref, torch.randn(2 * 70, 12), block_graphs(2, 70), None, dev)


@pytest.mark.parametrize("slope", [0.05, 0.8])
def test_tiled_negative_slope(dev, slope):
    mine, ref = twin_conv(12, 6, 3, False, 4, slope=slope, seed=8)
    ei = block_graphs(2, 90)
    _run(mine, ref, torch.randn(180, 12) * 3, ei, torch.randn(ei.size(1), 4), dev)


def test_tiled_attention_dropout(dev):
    """The tiled path's keep mask is [B, H, n, n] (drawn by torch)."""
    B, n, H, p = 2, 50, 4, 0.3
    mine, ref = twin_conv(10, 5, H, True, 3, dropout=p, seed=9)
    mine.train()
    ref.train()
    ei = block_graphs(B, n)
    torch.cuda.manual_seed(123)
    keep = (torch.rand(B, H, n, n, device=dev) >= p).to(torch.uint8).cpu()
    ref.attn_keep = dense_keep_to_edges(keep, ei, n)
    torch.cuda.manual_seed(123)
    _run(mine, ref, torch.randn(B * n, 10), ei, torch.randn(ei.size(1), 3), dev)


@pytest.mark.parametrize("act", ["relu", "tanh"])
def test_c5_stress_model(dev, act):
    """C5: n = 256, seq_length 4 (F = 1024, D = 12), 3 layers
    [16, 16, 16] x 8 heads concat, at batch 2 (the oracle's size)."""
    from spotv2net_amd import synthetic_batch
    n, S, B = 256, 4, 2
    mine, ref = twin_model(seed=5, num_node_features=n * S, num_edge_features=3 * S,
                           num_heads=8, output_node_channels=1, dim_hidden_layers=[16, 16, 16],
                           concat_heads=True, activation=act)
    ref64 = float64_twin(ref)
    data = synthetic_batch(B, S, n=n, seed=77)
    mine = mine.to(dev)
    out = mine(data.to(dev))
    rout = ref(data)

    class D64:
        x, edge_index, edge_attr = data.x.double(), data.edge_index, data.edge_attr.double()
    r64 = ref64(D64)
    w = torch.randn_like(rout)
    (out * w.to(dev)).sum().backward()
    (rout * w).sum().backward()
    (r64 * w.double()).sum().backward()
    assert_parity(out, rout, r64, what="forward")
    for (name, p), (_, q), (_, q64) in zip(mine.named_parameters(), ref.named_parameters(),
                                           ref64.named_parameters()):
        assert_parity(p.grad, q.grad, q64.grad, what=f"d{name}")


def test_c5_full_batch_runs(dev):
    """C5 at its full batch (1024 graphs, 67M edges): runs, finite, and the
    batch is the concatenation of independent graphs (graph 0 alone gives the
    same rows)."""
    from spotv2net_amd import Data, GATModel, synthetic_batch
    n, S, B = 256, 4, 1024
    E0 = n * (n - 1)
    torch.manual_seed(0)
    model = GATModel(n * S, 3 * S, 8, 1, [16, 16, 16], concat_heads=True).to(dev)
    data = synthetic_batch(B, S, n=n, seed=3, device=dev)
    with torch.no_grad():
        out = model(data)
        assert out.shape == (B * n,) and torch.isfinite(out).all()
        for g in (0, B - 1):
            one = Data(x=data.x[g * n:(g + 1) * n].clone(),
                       edge_index=data.edge_index[:, :E0].clone(),
                       edge_attr=data.edge_attr[g * E0:(g + 1) * E0].clone())
            torch.testing.assert_close(out[g * n:(g + 1) * n], model(one), rtol=1e-5, atol=1e-5)
