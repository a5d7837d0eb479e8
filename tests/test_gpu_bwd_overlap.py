"""The backward's side-stream overlap (stack.BWD_OVERLAP): the same kernels on
the same inputs, only on two streams, so gradients and trained parameters
must be bitwise those of the one-stream backward — eagerly (autograd) and in
a captured TrainStep."""
import copy

import pytest
import torch

from spotv2net_amd import stack

pytestmark = pytest.mark.gpu


def _model(dev, S, hidden, heads, seed, precision):
    from spotv2net_amd import GATModel
    torch.manual_seed(seed)
    m = GATModel(30 * S, 3 * S, heads, 1, list(hidden), concat_heads=True).to(dev)
    return m.set_precision(precision)


def _grads(model, data):
    model.zero_grad(set_to_none=True)
    out = model(data)
    loss = torch.nn.functional.mse_loss(out, data.y_x)
    loss.backward()
    torch.cuda.synchronize()
    return [p.grad.clone() for p in model.parameters()]


@pytest.mark.parametrize("precision,hidden", [("f32", (32, 16)), ("bf16", (48,)),
                                              ("f32", (16, 16, 8))])
def test_overlap_gradients_bitwise(dev, monkeypatch, precision, hidden):
    from spotv2net_amd import synthetic_batch
    data = synthetic_batch(64, 8, seed=11, device=dev)
    model = _model(dev, 8, hidden, 4, 3, precision)
    model.graph_replay = False
    monkeypatch.setattr(stack, "BWD_OVERLAP", "off")
    ref = _grads(model, data)
    monkeypatch.setattr(stack, "BWD_OVERLAP", "on")
    for _ in range(2):  # the second run reuses the side stream's pool
        got = _grads(model, data)
        for (n, _), a, b in zip(model.named_parameters(), ref, got):
            assert torch.equal(a, b), f"{precision} {hidden}: {n} differs with the overlap"


@pytest.mark.parametrize("precision,hidden", [("f32", (32, 16)), ("bf16", (48,))])
def test_overlap_trainstep_bitwise(dev, monkeypatch, precision, hidden):
    from spotv2net_amd import synthetic_batch
    from spotv2net_amd.train import TrainStep
    data = synthetic_batch(64, 8, seed=12, device=dev)
    m1 = _model(dev, 8, hidden, 4, 5, precision)
    m2 = copy.deepcopy(m1)
    monkeypatch.setattr(stack, "BWD_OVERLAP", "off")
    s1 = TrainStep(m1, data, lr=1e-2)
    monkeypatch.setattr(stack, "BWD_OVERLAP", "on")
    s2 = TrainStep(m2, data, lr=1e-2)  # captured with the fork / join
    for _ in range(4):
        l1, l2 = s1(), s2()
    torch.cuda.synchronize()
    assert torch.equal(l1, l2)
    for (n, p), (_, q) in zip(m1.named_parameters(), m2.named_parameters()):
        assert torch.equal(p, q), f"{precision} {hidden}: {n} differs with the overlap"
