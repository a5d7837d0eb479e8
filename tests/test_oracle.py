"""CPU tests that pin the oracle (oracle/): the PyG-2.3.0 op-for-op
restatement agrees with the independent dense float64 formulation, passes
float64 gradcheck and known-answer cases, and the reference-idiom dataset
restatement agrees with the product's batched window builder."""
import numpy as np
import pytest
import torch

from helpers import block_graphs


def _conv(in_ch, C, H, concat, edge_dim, seed=0, slope=0.2, dtype=torch.float64):
    from oracle.pyg_gatconv import OracleGATConv
    torch.manual_seed(seed)
    conv = OracleGATConv(in_ch, C, heads=H, concat=concat, edge_dim=edge_dim,
                         negative_slope=slope).to(dtype)
    with torch.no_grad():
        conv.bias.copy_(torch.randn_like(conv.bias) * 0.1)
    return conv


def _dense(conv, x, ei, ea, n):
    from oracle.dense import gat_layer_dense
    return gat_layer_dense(
        x.numpy(), ei.numpy(), None if ea is None else ea.numpy(),
        conv.lin_src.weight.detach().numpy(), conv.att_src.detach().numpy(),
        conv.att_dst.detach().numpy(),
        None if conv.lin_edge is None else conv.lin_edge.weight.detach().numpy(),
        None if conv.att_edge is None else conv.att_edge.detach().numpy(),
        conv.bias.detach().numpy(), conv.heads, conv.out_channels, conv.concat,
        conv.negative_slope, n)


@pytest.mark.parametrize("concat", [True, False])
@pytest.mark.parametrize("keep,shuffle,loops", [(1.0, False, False), (0.5, True, True)])
def test_pyg_restatement_matches_dense(concat, keep, shuffle, loops):
    n, B = 30, 2
    conv = _conv(12, 5, 3, concat, 4)
    torch.manual_seed(1)
    x = torch.randn(B * n, 12, dtype=torch.float64)
    ei = block_graphs(B, n, keep, shuffle, loops, seed=3)
    ea = torch.randn(ei.size(1), 4, dtype=torch.float64)
    out, (ei2, p) = conv(x, ei, ea, return_attention_weights=True)
    ref, P = _dense(conv, x, ei, ea, n)
    np.testing.assert_allclose(out.detach().numpy(), ref, rtol=1e-10, atol=1e-11)
    # attention weights of every (source -> target) edge incl. self loops
    src, dst = ei2
    g = dst // n
    Pd = P[g.numpy(), :, (dst - g * n).numpy(), (src - g * n).numpy()]
    np.testing.assert_allclose(p.detach().numpy(), Pd, rtol=1e-10, atol=1e-12)


def test_no_edge_attr_matches_dense():
    conv = _conv(6, 4, 2, True, 3)
    x = torch.randn(60, 6, dtype=torch.float64)
    ei = block_graphs(2, 30)
    out = conv(x, ei, None)
    ref, _ = _dense(conv, x, ei, None, 30)
    np.testing.assert_allclose(out.detach().numpy(), ref, rtol=1e-10, atol=1e-11)


def test_gradcheck_float64():
    conv = _conv(5, 3, 2, True, 2, seed=4)
    ei = block_graphs(2, 4, 0.8, True, True, seed=2)
    x = torch.randn(8, 5, dtype=torch.float64, requires_grad=True)
    ea = torch.randn(ei.size(1), 2, dtype=torch.float64)
    params = [p for p in conv.parameters()]
    torch.autograd.gradcheck(lambda x_, *ps: conv(x_, ei, ea), (x, *params), eps=1e-6,
                             atol=1e-7)


def test_known_answer_uniform_attention():
    """att_* = 0 => all logits 0 => uniform attention over the n in-edges
    (29 neighbours + self loop): out = mean of projected rows + bias."""
    n = 30
    conv = _conv(7, 4, 2, False, 3)
    with torch.no_grad():
        conv.att_src.zero_()
        conv.att_dst.zero_()
        conv.att_edge.zero_()
    x = torch.randn(n, 7, dtype=torch.float64)
    ei = block_graphs(1, n)
    out = conv(x, ei, torch.randn(ei.size(1), 3, dtype=torch.float64))
    xs = (x @ conv.lin_src.weight.t()).view(n, 2, 4)
    want = xs.mean(0, keepdim=True).expand(n, 2, 4).mean(1) + conv.bias
    torch.testing.assert_close(out, want, rtol=1e-12, atol=1e-12)


def test_known_answer_self_loop_mean_fill():
    """PyG add_self_loops(fill_value='mean') groups by TARGET: with one
    in-edge per target the loop's edge feature equals that edge's feature."""
    from oracle.pyg_gatconv import add_self_loops
    ei = torch.tensor([[0, 1, 2, 0], [1, 2, 0, 2]])
    ea = torch.tensor([[1.0], [2.0], [3.0], [5.0]])
    ei2, ea2 = add_self_loops(ei, ea, "mean", 3)
    assert ei2[:, -3:].tolist() == [[0, 1, 2], [0, 1, 2]]
    assert ea2[-3:, 0].tolist() == [3.0, 1.0, 3.5]


def test_dataset_restatement_matches_window_batch():
    """oracle.dataset (reference numpy idiom, utils/dataset.py:200-282) vs the
    product's batched builder and single-window builder."""
    from oracle.dataset import lagged_windows
    from spotv2net_amd import collate, window_batch, window_graph
    from spotv2net_amd.data import synthetic_series
    n, S, T = 6, 3, 9
    V, W = synthetic_series(T, n, seed=2, dtype=torch.float64)
    ref = lagged_windows(list(V.numpy()), list(W.numpy()), S)
    assert len(ref) == T - S
    b = window_batch(V, W, torch.arange(T - S), S)
    c = collate([window_graph(V[i:i + S + 1], W[i:i + S + 1]) for i in range(T - S)])
    off = 0
    for k, r in enumerate(ref):
        assert torch.equal(b.x[k * n:(k + 1) * n], r["x"])
        assert torch.equal(c.x[k * n:(k + 1) * n], r["x"])
        E0 = n * (n - 1)
        assert torch.equal(b.edge_attr[k * E0:(k + 1) * E0], r["edge_attr"])
        assert torch.equal(c.edge_attr[k * E0:(k + 1) * E0], r["edge_attr"])
        assert torch.equal(b.edge_index[:, k * E0:(k + 1) * E0] - off, r["edge_index"])
        assert torch.equal(b.y_x[k * n:(k + 1) * n], r["y_x"])
        off += n
    assert torch.equal(b.edge_index, c.edge_index)


def test_canonical_pairs_match_reference_argwhere():
    from spotv2net_amd.layout import canonical_pairs
    n = 30
    mask = np.triu(np.ones((n, n)), k=1) > 0
    up = np.argwhere(mask).T
    s, t = canonical_pairs(n)
    assert s[:435] == up[0].tolist() and t[:435] == up[1].tolist()
    assert s[435:] == up[1].tolist() and t[435:] == up[0].tolist()
