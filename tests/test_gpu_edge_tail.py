"""The edge-logit weight gradient fused into layer 0's n <= 32 attention
backward (sv2n_gat_attn_bwd_edge, ABI 12) — the backward of PyG GATConv's
lin_edge / att_edge (reference utils/models.py:146) for every layer, with
edge_attr streamed inside the attention kernel instead of by a separate
edge-gradient pass.

Checked against the separate pass (sv2n_edge_logits_bwd: same products,
another summation order) and against the PyG-semantics oracle (tolerance of
tests/helpers.py); every other gradient is bit-identical between the paths."""
import copy

import pytest
import torch

from helpers import assert_close, assert_parity, float64_twin, twin_model

pytestmark = pytest.mark.gpu


def _canonical(data, n=30):
    from spotv2net_amd import Batch
    return Batch(x=data.x, edge_index=data.edge_index, edge_attr=data.edge_attr, y_x=data.y_x,
                 batch=data.batch, ptr=data.ptr, nodes_per_graph=n, canonical_edges=True)


def _grads(model, data, tail, seed=0):
    from spotv2net_amd import stack
    old, old_cv = stack.EDGE_TAIL, stack.COV_VAR_EDGES
    stack.EDGE_TAIL = tail
    stack.COV_VAR_EDGES = "off"  # the tail is an alternative to the generic edge-row passes
    try:
        model.zero_grad()
        torch.cuda.manual_seed(seed)
        loss = torch.nn.functional.mse_loss(model(_canonical(data)), data.y_x)
        loss.backward()
        torch.cuda.synchronize()
        used = stack.LAST_PATH["edge_tail"]
    finally:
        stack.EDGE_TAIL, stack.COV_VAR_EDGES = old, old_cv
    return {n: p.grad.detach().clone() for n, p in model.named_parameters()}, used


@pytest.mark.parametrize("S,heads,hidden,concat,B,dropout", [
    (4, 4, [16, 8], True, 24, 0.0),     # C2's structure (2 layers x 4 heads: 8 columns)
    (2, 1, [20], False, 16, 0.0),       # C1's structure (1 layer, 1 head; even D)
    (2, 2, [12, 6, 5], True, 9, 0.0),   # 3 layers x 2 heads (6 of 8 columns)
    (4, 4, [16, 8], True, 20, 0.2),     # post-layer dropout (its draws in the kernel)
])
def test_edge_tail_matches_separate_pass(dev, S, heads, hidden, concat, B, dropout):
    from spotv2net_amd import GATModel, synthetic_batch
    torch.manual_seed(11)
    m1 = GATModel(30 * S, 3 * S, heads, 1, hidden, concat_heads=concat, dropout=dropout).to(dev)
    m1.graph_replay = False
    m2 = copy.deepcopy(m1)
    data = synthetic_batch(B, S, seed=5, device=dev)
    g1, used1 = _grads(m1, data, "on", seed=3)
    g2, used2 = _grads(m2, data, "off", seed=3)
    assert used1 is True and used2 is False
    for name in g1:
        if "lin_edge" in name or "att_edge" in name:
            assert_close(g1[name], g2[name], what=name)
        else:
            assert torch.equal(g1[name], g2[name]), name


def test_edge_tail_c2_shape_matches_oracle(dev):
    """C2's model (S 42: D = 126, GAT [100, 50] x 4 heads concat) at B = 48:
    the fused edge gradients by the parity rule against the oracle."""
    from spotv2net_amd import Data, synthetic_batch
    S = 42
    mine, ref = twin_model(seed=5154, num_node_features=30 * S, num_edge_features=3 * S,
                           num_heads=4, output_node_channels=1, dim_hidden_layers=[100, 50],
                           concat_heads=True)
    ref64 = float64_twin(ref)
    mine = mine.to(dev)
    mine.graph_replay = False
    cpu = synthetic_batch(48, S, seed=1234)
    g, used = _grads(mine, cpu.to(dev), "on")
    assert used is True
    d = Data(x=cpu.x, edge_index=cpu.edge_index, edge_attr=cpu.edge_attr)
    torch.nn.functional.mse_loss(ref(d), cpu.y_x).backward()
    d64 = Data(x=cpu.x.double(), edge_index=cpu.edge_index, edge_attr=cpu.edge_attr.double())
    torch.nn.functional.mse_loss(ref64(d64), cpu.y_x.double()).backward()
    for (name, q), (_, q64) in zip(ref.named_parameters(), ref64.named_parameters()):
        if "lin_edge" in name or "att_edge" in name:
            assert_parity(g[name], q.grad, q64.grad, what=f"d{name}")


def test_edge_tail_deterministic(dev):
    """Fixed-order sums: two backwards give the same bits."""
    from spotv2net_amd import GATModel, synthetic_batch
    torch.manual_seed(2)
    m = GATModel(30 * 4, 12, 4, 1, [16, 8], concat_heads=True).to(dev)
    m.graph_replay = False
    data = synthetic_batch(40, 4, seed=9, device=dev)
    a, _ = _grads(m, data, "on")
    b, _ = _grads(m, data, "on")
    for k in a:
        assert torch.equal(a[k], b[k]), k

