"""The fused nodes return their parameter gradients to autograd: hooks,
torch.autograd.grad and DistributedDataParallel see them (the reference's
caller, 5_train_SpotV2Net.py:150-159, is what a user would wrap in DDP)."""
import copy
import os
import socket

import pytest
import torch

from helpers import assert_close

pytestmark = pytest.mark.gpu


def _model(dev, seed=0, **kw):
    from spotv2net_amd import GATModel
    torch.manual_seed(seed)
    return GATModel(30 * 4, 3 * 4, 4, 1, [16, 8], concat_heads=True, **kw).to(dev)


def test_autograd_grad_returns_parameter_grads(dev):
    from spotv2net_amd import synthetic_batch
    m = _model(dev, seed=1)
    data = synthetic_batch(5, 4, seed=2, device=dev)
    params = list(m.parameters())
    loss = torch.nn.functional.mse_loss(m(data), data.y_x)
    grads = torch.autograd.grad(loss, params)
    assert all(g is not None for g in grads)
    assert all(p.grad is None for p in params), "autograd.grad must not touch .grad"
    loss2 = torch.nn.functional.mse_loss(m(data), data.y_x)
    loss2.backward()
    for (name, p), g in zip(m.named_parameters(), grads):
        assert torch.equal(p.grad, g), name


def test_parameter_hooks_fire(dev):
    from spotv2net_amd import synthetic_batch
    m = _model(dev, seed=2)
    seen = []
    for name, p in m.named_parameters():
        p.register_hook(lambda g, name=name: seen.append(name))
    data = synthetic_batch(3, 4, seed=3, device=dev)
    m.mse_loss(data).backward()
    assert sorted(seen) == sorted(n for n, _ in m.named_parameters())


def test_backward_inputs_only_leaves_param_grads(dev):
    """backward(inputs=[x]) must not write parameter gradients."""
    from spotv2net_amd import synthetic_batch
    m = _model(dev, seed=3)
    data = synthetic_batch(3, 4, seed=4, device=dev)
    x = data.x.clone().requires_grad_(True)
    data.x = x
    m(data).sum().backward(inputs=[x])
    assert x.grad is not None
    assert all(p.grad is None for p in m.parameters())


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_ddp_world1_trains_like_trainstep(dev):
    """DistributedDataParallel(GATModel) over RCCL (world size 1) with
    torch.optim.Adam, two reference-loop steps, equals TrainStep (fused Adam,
    direct gradient accumulation) for the same two steps."""
    import torch.distributed as dist
    from torch.nn.parallel import DistributedDataParallel as DDP

    from spotv2net_amd import synthetic_batch
    from spotv2net_amd.train import TrainStep
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0,
                            world_size=1, device_id=dev)
    try:
        m1 = _model(dev, seed=4)
        m2 = copy.deepcopy(m1)
        data = synthetic_batch(12, 4, seed=5, device=dev)
        ddp = DDP(m1, device_ids=[dev.index])
        opt = torch.optim.Adam(ddp.parameters(), lr=1e-3)
        for _ in range(2):
            loss = torch.nn.functional.mse_loss(ddp(data), data.y_x)
            opt.zero_grad()
            loss.backward()
            opt.step()
        step = TrainStep(m2, data, lr=1e-3, use_graph=False)
        for _ in range(2):
            step()
        torch.cuda.synchronize()
        for (n, p), (_, q) in zip(m1.named_parameters(), m2.named_parameters()):
            assert_close(p, q, tol=1e-6, what=n)
    finally:
        dist.destroy_process_group()


def test_pyg_linear_module(dev):
    """spotv2net_amd.Linear (PyG's bias-free glorot Linear that GATConv holds)
    used standalone: f32 MFMA forward and both backward products."""
    from spotv2net_amd import Linear
    torch.manual_seed(6)
    lin = Linear(70, 33).to(dev)
    x = torch.randn(257, 70, device=dev, requires_grad=True)
    w = torch.randn(257, 33, device=dev)
    (lin(x) * w).sum().backward()
    xr = x.detach().cpu().double().requires_grad_(True)
    wr = lin.weight.detach().cpu().double().requires_grad_(True)
    (torch.nn.functional.linear(xr, wr) * w.cpu().double()).sum().backward()
    assert_close(lin(x), torch.nn.functional.linear(xr, wr), what="fwd")
    assert_close(x.grad, xr.grad, what="dx")
    assert_close(lin.weight.grad, wr.grad, what="dW")
