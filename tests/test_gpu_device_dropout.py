"""Device dropout generator of the captured training step (ABI 17,
sv2n_dropout_uniform; stack.device_dropout, train.TrainStep): the uniforms
bit-exact against the numpy restatement (tests/philox_ref.py), the mask
statistics, graph replay == eager steps, and one training step's loss and
gradients against the oracle with the masks rebuilt on the host (post-layer
dropout, utils/models.py:148, tolerance of tests/helpers.py)."""
import copy

import numpy as np
import pytest
import torch

from helpers import assert_close, assert_parity, float64_twin, twin_model
from philox_ref import dropout_uniform_ref

import spotv2net_amd  # noqa: F401  (registers torch.ops.sv2n)

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("rows,cols,seed,step,salt", [
    (3840, 500, 5154, 0, 0), (7, 5, 2 ** 40 + 3, 12, 1), (1, 1, 0, 3, 2), (30, 400, 9, 1000, 0),
])
def test_uniforms_match_restatement(dev, rows, cols, seed, step, salt):
    st = torch.full((1,), float(step), device=dev)
    u = torch.ops.sv2n.dropout_uniform(rows, cols, st, seed, salt)
    want = dropout_uniform_ref(rows * cols, seed, step, salt).reshape(rows, cols)
    assert np.array_equal(u.cpu().numpy(), want)


def test_seed_at_or_above_2_63(dev):
    """torch.seed() draws any 64-bit value; TrainStep's default dropout seed
    is torch.initial_seed(), so a seed >= 2**63 must run (folded into the
    op's int64 argument, reinterpreted as uint64: the restatement's draws)."""
    from spotv2net_amd import GATModel, synthetic_batch
    from spotv2net_amd.stack import _int64_seed
    from spotv2net_amd.train import TrainStep
    big = 2 ** 63 + 5
    st = torch.full((1,), 2.0, device=dev)
    u = torch.ops.sv2n.dropout_uniform(30, 40, st, _int64_seed(big), 1)
    assert np.array_equal(u.cpu().numpy(), dropout_uniform_ref(1200, big, 2, 1).reshape(30, 40))
    torch.manual_seed(big)
    assert torch.initial_seed() == big
    m = GATModel(120, 12, 4, 1, [16, 8], dropout=0.2, concat_heads=True).to(dev)
    data = synthetic_batch(8, 4, seed=3, device=dev)
    step = TrainStep(m, data, lr=1e-3, use_graph=True)
    assert step.device_rng and step.dropout_seed == big
    losses = [float(step()) for _ in range(2)]
    assert all(np.isfinite(losses)), losses


def test_mask_statistics(dev):
    st = torch.zeros(1, device=dev)
    u = torch.ops.sv2n.dropout_uniform(4096, 1000, st, 77, 0)
    for p in (0.1, 0.5):
        keep = (u >= p).float().mean().item()
        assert abs(keep - (1 - p)) < 2e-3, (p, keep)
    st += 1
    assert not torch.equal(u, torch.ops.sv2n.dropout_uniform(4096, 1000, st, 77, 0))


def test_trainstep_replay_equals_eager_with_dropout(dev):
    """the captured step (no torch random op inside) == eager steps, bit for
    bit, with post-layer dropout on both layers and the fused head."""
    from spotv2net_amd import GATModel, synthetic_batch
    from spotv2net_amd.train import TrainStep
    torch.manual_seed(4)
    m1 = GATModel(120, 12, 4, 1, [16, 8], dropout=0.2, concat_heads=True).to(dev)
    m2 = copy.deepcopy(m1)
    data = synthetic_batch(24, 4, seed=3, device=dev)
    s1 = TrainStep(m1, data, lr=1e-3, use_graph=True, dropout_seed=99)
    s2 = TrainStep(m2, data, lr=1e-3, use_graph=False, dropout_seed=99)
    assert s1.device_rng and s2.device_rng
    for _ in range(4):
        a, b = float(s1()), float(s2())
        assert a == b, (a, b)
    for (n, p), (_, q) in zip(m1.named_parameters(), m2.named_parameters()):
        assert torch.equal(p, q), n


def test_device_dropout_step_matches_oracle(dev):
    """one training forward + MSE backward under device_dropout (the fused
    head + loss path the TrainStep takes) against the oracle fed the same
    keep masks, rebuilt from the restatement: salt = layer, step = the
    optimizer's step count."""
    from spotv2net_amd import Data, synthetic_batch
    from spotv2net_amd.stack import device_dropout, direct_grad_accumulation
    S, B, p, seed, step = 2, 16, 0.1, 2024, 5
    mine, ref = twin_model(seed=11, num_node_features=30 * S, num_edge_features=3 * S,
                           num_heads=6, output_node_channels=1, dim_hidden_layers=[40, 20],
                           dropout=p, concat_heads=True, activation="tanh")
    ref64 = float64_twin(ref)
    mine = mine.to(dev)
    data = synthetic_batch(B, S, seed=8)
    gd = data.to(dev)
    N = data.x.shape[0]
    keep = [torch.from_numpy(dropout_uniform_ref(N * oc, seed, step, salt).reshape(N, oc) >= p)
            for salt, oc in enumerate((6 * 40, 20))]  # the last layer averages its heads
    ref.post_keep = keep
    ref64.post_keep = keep
    for q in mine.parameters():
        q.grad = torch.zeros_like(q)
    st = torch.full((1,), float(step), device=dev)
    with device_dropout(seed, st), direct_grad_accumulation():
        loss = mine._train_head_mse(gd, gd.y_x)
    assert loss is not None, "the fused head path must take this shape"
    d = Data(x=data.x, edge_index=data.edge_index, edge_attr=data.edge_attr)
    rl = torch.nn.functional.mse_loss(ref(d), data.y_x)
    rl.backward()
    r64 = torch.nn.functional.mse_loss(
        ref64(Data(x=data.x.double(), edge_index=data.edge_index,
                   edge_attr=data.edge_attr.double())), data.y_x.double())
    r64.backward()
    assert_parity(loss, rl, r64, what="loss")
    for (name, q), (_, r), (_, r64q) in zip(mine.named_parameters(), ref.named_parameters(),
                                          ref64.named_parameters()):
        assert_parity(q.grad, r.grad, r64q.grad, what=f"d{name}")


def test_unfused_path_draws_the_same_masks(dev):
    """model(data) + MSE under device_dropout == the fused head path under
    the same key (both draw through stack._post_uniforms)."""
    from spotv2net_amd import GATModel, synthetic_batch
    from spotv2net_amd.stack import HEAD_FUSE, device_dropout, direct_grad_accumulation
    assert HEAD_FUSE == "on"
    torch.manual_seed(21)
    m1 = GATModel(60, 6, 4, 1, [16, 8], dropout=0.3, concat_heads=True).to(dev)
    m2 = copy.deepcopy(m1)
    data = synthetic_batch(12, 2, seed=6, device=dev)
    st = torch.full((1,), 3.0, device=dev)
    for q in m1.parameters():
        q.grad = torch.zeros_like(q)
    with device_dropout(17, st), direct_grad_accumulation():
        l1 = m1._train_head_mse(data, data.y_x)
    with device_dropout(17, st):
        l2 = torch.nn.functional.mse_loss(m2(data), data.y_x)
        l2.backward()
    assert_close(l1, l2, tol=1e-6, what="loss")
    for (n, p), (_, q) in zip(m1.named_parameters(), m2.named_parameters()):
        assert_close(p.grad, q.grad, what=n)
