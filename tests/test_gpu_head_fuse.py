"""The training step's output head + MSE fused into the last GAT layer's
attention forward (sv2n_gat_attn_fwd_head_mse, ABI 13): GATModel.linear
(reference utils/models.py:120, :150) and nn.MSELoss with loss.backward()
(5_train_SpotV2Net.py:125, :150-158) computed where the last layer's output
is produced.

Checked against the unfused product path (separate head + loss launch: same
products, other summation orders) and, at the bench's C2 size, against the
PyG-semantics oracle by the parity rule of tests/helpers.py."""
import copy

import pytest
import torch

from helpers import assert_close, assert_parity, float64_twin, twin_model

pytestmark = pytest.mark.gpu


def _step(model, data, fuse):
    """zero grads, one fused (or unfused) training forward + backward; the
    loss and every parameter gradient"""
    from spotv2net_amd import stack
    old = stack.HEAD_FUSE
    stack.HEAD_FUSE = fuse
    try:
        for p in model.parameters():
            p.grad = torch.zeros_like(p)
        loss = model._train_head_mse(data, data.y_x)
        if loss is None:
            loss = None
        torch.cuda.synchronize()
    finally:
        stack.HEAD_FUSE = old
    return loss, {n: p.grad.detach().clone() for n, p in model.named_parameters()}


def _unfused(model, data):
    for p in model.parameters():
        p.grad = None
    loss = torch.nn.functional.mse_loss(model(data), data.y_x)
    loss.backward()
    torch.cuda.synchronize()
    return loss.detach(), {n: p.grad.detach().clone() for n, p in model.named_parameters()}


@pytest.mark.parametrize("S,heads,hidden,concat,B,act,dropout,dropout_att", [
    (4, 4, [16, 8], True, 24, "relu", 0.0, 0.0),     # C2's structure (last layer: head mean)
    (2, 1, [20], False, 16, "relu", 0.0, 0.0),       # C1's structure (one layer)
    (2, 3, [12, 6, 5], True, 9, "tanh", 0.0, 0.0),   # three layers, tanh
    (4, 4, [16, 8], True, 20, "relu", 0.2, 0.1),     # post-layer and attention dropout
    (2, 6, [40], True, 12, "sigmoid", 0.1, 0.0),     # C3's structure (one layer, 6 heads)
])
def test_fused_head_matches_unfused(dev, S, heads, hidden, concat, B, act, dropout, dropout_att):
    from spotv2net_amd import GATModel, synthetic_batch
    torch.manual_seed(21)
    m1 = GATModel(30 * S, 3 * S, heads, 1, hidden, concat_heads=concat, activation=act,
                  dropout=dropout, dropout_att=dropout_att).to(dev)
    m1.graph_replay = False
    m2 = copy.deepcopy(m1)
    data = synthetic_batch(B, S, seed=6, device=dev)
    torch.cuda.manual_seed(9)
    l1, g1 = _step(m1, data, "on")
    assert l1 is not None, "the fused path must take this shape"
    torch.cuda.manual_seed(9)  # same draws (attention keep masks, post-layer uniforms)
    l2, g2 = _unfused(m2, data)
    assert_close(l1, l2, tol=1e-6, what="loss")
    for name in g1:
        assert_close(g1[name], g2[name], what=name)


def test_fused_head_off_switch_and_fallbacks(dev):
    """HEAD_FUSE = "off", multi-output heads and standardize fall back (None)."""
    from spotv2net_amd import GATModel, synthetic_batch
    torch.manual_seed(3)
    data = synthetic_batch(8, 2, seed=2, device=dev)
    m = GATModel(60, 6, 2, 1, [8], concat_heads=True).to(dev)
    assert _step(m, data, "off")[0] is None
    m2 = GATModel(60, 6, 2, 3, [8], concat_heads=True).to(dev)   # output_node_channels 3
    assert m2._train_head_mse(data, data.y_x.repeat_interleave(3)) is None


def test_fused_head_c2_full_batch_matches_oracle(dev):
    """C2 at the bench's B = 512: the fused step's loss and every gradient
    (head included) against the oracle, relu sides injected as in
    test_gpu_parity_full."""
    from spotv2net_amd import Data, synthetic_batch
    from test_gpu_parity_full import _check_kinks, _relu_masks
    S = 42
    mine, ref = twin_model(seed=5154, num_node_features=30 * S, num_edge_features=3 * S,
                           num_heads=4, output_node_channels=1, dim_hidden_layers=[100, 50],
                           concat_heads=True)
    ref64 = float64_twin(ref)
    mine = mine.to(dev)
    data = synthetic_batch(512, S, seed=1234)
    gd = data.to(dev)
    masks = _relu_masks(mine, gd)
    ref.act_masks = masks
    ref64.act_masks = masks
    loss, grads = _step(mine, gd, "on")
    assert loss is not None
    d = Data(x=data.x, edge_index=data.edge_index, edge_attr=data.edge_attr)
    rl = torch.nn.functional.mse_loss(ref(d), data.y_x)
    rl.backward()
    r64 = torch.nn.functional.mse_loss(
        ref64(Data(x=data.x.double(), edge_index=data.edge_index,
                   edge_attr=data.edge_attr.double())), data.y_x.double())
    r64.backward()
    _check_kinks(ref64, masks)
    assert_parity(loss, rl, r64, what="loss")
    for (name, q), (_, q64) in zip(ref.named_parameters(), ref64.named_parameters()):
        assert_parity(grads[name], q.grad, q64.grad, what=f"d{name}")


def test_trainstep_takes_the_fused_head(dev):
    """TrainStep (graph replay) runs the fused path and equals its eager
    unfused twin step for step within rounding."""
    from spotv2net_amd import GATModel, stack, synthetic_batch
    from spotv2net_amd.train import TrainStep
    torch.manual_seed(8)
    m1 = GATModel(120, 12, 4, 1, [16, 8], concat_heads=True).to(dev)
    m2 = copy.deepcopy(m1)
    data = synthetic_batch(32, 4, seed=5, device=dev)
    s1 = TrainStep(m1, data, lr=1e-3, use_graph=True)
    old = stack.HEAD_FUSE
    stack.HEAD_FUSE = "off"
    try:
        s2 = TrainStep(m2, data, lr=1e-3, use_graph=False)
        losses = []
        for _ in range(3):
            a = s1()
            b = s2()
            losses.append((float(a), float(b)))
    finally:
        stack.HEAD_FUSE = old
    for a, b in losses:
        assert abs(a - b) <= 1e-5 * max(1.0, abs(b)), losses
    for (n, p), (_, q) in zip(m1.named_parameters(), m2.named_parameters()):
        assert_close(p, q, tol=1e-5, what=n)
