"""GPU parity of the edge-fused attention (sv2n_attn_fused.hip: edge logits
computed inside the attention for 32 < n <= 256 and narrow edge_attr, the C5
shapes of SURVEY.md §8d) against the PyG-2.3.0 restatement, and against the
planes path (edge pass + sv2n_attn_tiled.hip) on the same inputs.  Tolerance:
tests/helpers.py (1e-5 scaled by max(1, |ref|))."""
import pytest
import torch

from helpers import (assert_close, assert_parity, block_graphs, dense_keep_to_edges,
                     float64_twin, twin_conv, twin_model)
from test_gpu_conv import _run

pytestmark = pytest.mark.gpu


@pytest.fixture
def edge_mode():
    from spotv2net_amd import stack
    prev = stack.EDGE_FUSED

    def set_mode(m):
        stack.EDGE_FUSED = m
    yield set_mode
    stack.EDGE_FUSED = prev


def _path():
    from spotv2net_amd import stack
    return stack.LAST_PATH["attention"]


@pytest.mark.parametrize("n,H,C,D,concat", [(33, 8, 16, 12, True), (64, 3, 8, 6, False),
                                            (100, 1, 4, 3, True), (256, 8, 16, 12, False),
                                            (200, 5, 12, 12, True), (47, 2, 16, 3, False)])
def test_fused_matches_oracle(dev, n, H, C, D, concat):
    B = 2
    mine, ref = twin_conv(20, C, H, concat, D, seed=n + H)
    torch.manual_seed(n)
    ei = block_graphs(B, n)
    _run(mine, ref, torch.randn(B * n, 20), ei, torch.randn(ei.size(1), D), dev)
    assert _path() == "fused"


@pytest.mark.parametrize("n,keep_frac,shuffle,loops", [(64, 1.0, True, False),
                                                       (100, 0.5, True, True),
                                                       (256, 0.3, False, True)])
def test_fused_block_layouts(dev, n, keep_frac, shuffle, loops):
    """Edge-id maps (any order, missing edges, input self loops, a target with
    no in-edges) on the fused kernels."""
    B = 2
    mine, ref = twin_conv(10, 8, 4, True, 6, seed=7)
    ei = block_graphs(B, n, keep_frac, shuffle, loops, seed=n)
    ei = ei[:, ei[1] != n + 3]
    _run(mine, ref, torch.randn(B * n, 10), ei, torch.randn(ei.size(1), 6), dev)
    assert _path() == "fused"


@pytest.mark.parametrize("slope", [0.05, 0.8])
def test_fused_negative_slope(dev, slope):
    mine, ref = twin_conv(12, 8, 3, False, 3, slope=slope, seed=8)
    ei = block_graphs(2, 90)
    _run(mine, ref, torch.randn(180, 12) * 3, ei, torch.randn(ei.size(1), 3), dev)
    assert _path() == "fused"


def test_fused_attention_dropout(dev):
    B, n, H, p = 2, 50, 4, 0.3
    mine, ref = twin_conv(10, 8, H, True, 6, dropout=p, seed=9)
    mine.train()
    ref.train()
    ei = block_graphs(B, n)
    torch.cuda.manual_seed(123)
    keep = (torch.rand(B, H, n, n, device=dev) >= p).to(torch.uint8).cpu()
    ref.attn_keep = dense_keep_to_edges(keep, ei, n)
    torch.cuda.manual_seed(123)
    _run(mine, ref, torch.randn(B * n, 10), ei, torch.randn(ei.size(1), 6), dev)
    assert _path() == "fused"


def _conv_grads(conv, x, ei, ea, w):
    conv.zero_grad()
    xg = x.clone().requires_grad_(True)
    out = conv(xg, ei, ea)
    (out * w).sum().backward()
    return [out.detach().clone(), xg.grad.clone()] + [p.grad.clone() for p in conv.parameters()]


def test_fused_equals_planes_path(dev, edge_mode):
    """The fused kernels and the edge pass + tiled kernels agree on the same
    inputs (C5 layer shape: n 256, D 12, 8 heads x 16)."""
    B, n = 2, 256
    mine, _ = twin_conv(64, 16, 8, True, 12, seed=11)
    mine = mine.to(dev)
    torch.manual_seed(3)
    ei = block_graphs(B, n).to(dev)
    x = torch.randn(B * n, 64, device=dev)
    ea = torch.randn(ei.size(1), 12, device=dev)
    w = torch.randn(B * n, 128, device=dev)
    edge_mode("on")
    a = _conv_grads(mine, x, ei, ea, w)
    assert _path() == "fused"
    edge_mode("off")
    b = _conv_grads(mine, x, ei, ea, w)
    assert _path() == "tiled"
    for u, v in zip(a, b):
        assert_close(u, v, what="fused vs planes")


def test_fused_deterministic(dev):
    """No atomics: two backward passes give bit-identical gradients."""
    B, n = 3, 128
    mine, _ = twin_conv(32, 16, 8, True, 12, seed=12)
    mine = mine.to(dev)
    torch.manual_seed(4)
    ei = block_graphs(B, n).to(dev)
    x = torch.randn(B * n, 32, device=dev)
    ea = torch.randn(ei.size(1), 12, device=dev)
    w = torch.randn(B * n, 128, device=dev)
    a = _conv_grads(mine, x, ei, ea, w)
    b = _conv_grads(mine, x, ei, ea, w)
    for u, v in zip(a, b):
        assert torch.equal(u, v)


@pytest.mark.parametrize("concat", [True, False])
def test_fused_three_layer_model(dev, concat):
    """A 3-layer GATModel (utils/models.py:86-152) on 64-node graphs with
    seq_length 2 (D 6): every layer on the fused kernels, MSE backward."""
    from spotv2net_amd import synthetic_batch
    n, S, B = 64, 2, 3
    mine, ref = twin_model(seed=21, num_node_features=n * S, num_edge_features=3 * S,
                           num_heads=4, output_node_channels=1, dim_hidden_layers=[8, 8, 8],
                           concat_heads=concat, activation="tanh")
    ref64 = float64_twin(ref)
    data = synthetic_batch(B, S, n=n, seed=5)
    mine = mine.to(dev)
    out = mine(data.to(dev))
    assert _path() == "fused"
    rout = ref(data)

    class D64:
        x, edge_index, edge_attr = data.x.double(), data.edge_index, data.edge_attr.double()
    r64 = ref64(D64)
    y = torch.randn_like(rout)
    torch.nn.functional.mse_loss(out, y.to(dev)).backward()
    torch.nn.functional.mse_loss(rout, y).backward()
    torch.nn.functional.mse_loss(r64, y.double()).backward()
    assert_parity(out, rout, r64, what="forward")
    for (name, p), (_, q), (_, q64) in zip(mine.named_parameters(), ref.named_parameters(),
                                           ref64.named_parameters()):
        assert_parity(p.grad, q.grad, q64.grad, what=f"d{name}")


def test_fused_eval_forward_saves_nothing(dev):
    """Inference (no grad): the fused forward writes no statistics and matches
    the training-mode output."""
    mine, _ = twin_conv(16, 16, 8, True, 12, seed=13)
    mine = mine.to(dev).eval()
    ei = block_graphs(2, 80).to(dev)
    x = torch.randn(160, 16, device=dev)
    ea = torch.randn(ei.size(1), 12, device=dev)
    with torch.no_grad():
        a = mine(x, ei, ea)
    b = mine(x.clone().requires_grad_(True), ei, ea).detach()
    assert torch.equal(a, b)
