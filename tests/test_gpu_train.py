"""Training-step runtime on the GPU: sv2n Adam vs torch.optim.Adam, hipGraph
replay vs eager, and loss decrease on the C2 model."""
import copy

import pytest
import torch

from helpers import assert_close

pytestmark = pytest.mark.gpu


def _model(dev, S=4, hidden=(16, 8), heads=4, seed=0, **kw):
    from spotv2net_amd import GATModel
    torch.manual_seed(seed)
    return GATModel(30 * S, 3 * S, heads, 1, list(hidden), concat_heads=True, **kw).to(dev)


def test_flat_adam_matches_torch_adam(dev):
    from spotv2net_amd import synthetic_batch
    from spotv2net_amd.train import TrainStep
    data = synthetic_batch(8, 4, seed=1, device=dev)
    m1 = _model(dev)
    m2 = copy.deepcopy(m1)
    s1 = TrainStep(m1, data, lr=1e-2, use_graph=False, optimizer="sv2n")
    s2 = TrainStep(m2, data, lr=1e-2, use_graph=False, optimizer="torch")
    for _ in range(5):
        s1()
        s2()
    for (n, p), (_, q) in zip(m1.named_parameters(), m2.named_parameters()):
        assert_close(p, q, tol=2e-5, what=n)


def test_graph_replay_equals_eager(dev):
    from spotv2net_amd import synthetic_batch
    from spotv2net_amd.train import TrainStep
    data = synthetic_batch(16, 4, seed=2, device=dev)
    m1 = _model(dev, seed=3)
    m2 = copy.deepcopy(m1)
    s1 = TrainStep(m1, data, use_graph=True, warmup=3)  # warm-up is undone after capture
    s2 = TrainStep(m2, data, use_graph=False)
    for (n, p), (_, q) in zip(m1.named_parameters(), m2.named_parameters()):
        assert torch.equal(p, q), f"{n}: constructing a TrainStep must not train"
    for _ in range(4):
        s1()
        s2()
    torch.cuda.synchronize()
    for (n, p), (_, q) in zip(m1.named_parameters(), m2.named_parameters()):
        assert torch.allclose(p, q, rtol=0, atol=1e-6), n


def test_c2_loss_decreases(dev):
    from spotv2net_amd import GATModel, synthetic_batch
    from spotv2net_amd.train import TrainStep
    torch.manual_seed(5154)
    model = GATModel(1260, 126, 4, 1, [100, 50], concat_heads=True).to(dev)
    data = synthetic_batch(128, 42, seed=3, device=dev)
    step = TrainStep(model, data, lr=1e-3)
    first = float(step().item())
    for _ in range(30):
        step()
    last = float(step().item())
    assert last < first, (first, last)


def test_dropout_training_runs_and_is_seeded(dev):
    """dropout / dropout_att > 0 (yaml C3 uses dropout 0.1): train mode is
    stochastic, eval mode deterministic, gradients finite."""
    from spotv2net_amd import synthetic_batch
    m = _model(dev, dropout=0.3, dropout_att=0.2)
    data = synthetic_batch(6, 4, seed=4, device=dev)
    m.train()
    torch.manual_seed(7)
    a = m(data)
    torch.manual_seed(7)
    b = m(data)
    c = m(data)
    assert torch.equal(a, b) and not torch.equal(a, c)
    (a ** 2).mean().backward()
    for p in m.parameters():
        assert p.grad is not None and torch.isfinite(p.grad).all()
    m.eval()
    with torch.no_grad():
        assert torch.equal(m(data), m(data))


@pytest.mark.parametrize("out_ch", [1, 3, 14])
def test_fused_head_mse_matches_unfused(dev, out_ch):
    """GATModel.mse_loss (sv2n_head_mse_fwd/bwd) == nn.MSELoss()(model(data), y)
    (reference 5_train_SpotV2Net.py:125, :154), loss and every gradient;
    an upstream gradient scale (2·loss) is honoured."""
    from spotv2net_amd import GATModel, synthetic_batch
    torch.manual_seed(1)
    m1 = GATModel(120, 12, 4, out_ch, [16, 8], concat_heads=True).to(dev)
    m2 = copy.deepcopy(m1)
    data = synthetic_batch(6, 4, seed=5, device=dev)
    y = torch.randn(data.x.shape[0] * out_ch, device=dev)
    l1 = m1.mse_loss(data, y)
    (2.0 * l1).backward()
    l2 = torch.nn.functional.mse_loss(m2(data), y)
    (2.0 * l2).backward()
    assert_close(l1, l2, tol=1e-6, what="loss")
    for (n, p), (_, q) in zip(m1.named_parameters(), m2.named_parameters()):
        assert_close(p.grad, q.grad, tol=1e-6, what=n)


@pytest.mark.parametrize("out_ch,rows,C", [(1, 15360, 50), (3, 180, 50), (14, 1000, 50),
                                           (1, 3840, 500), (4, 1001, 500), (2, 777, 130)])
def test_head_mse_train_matches_fwd_bwd(dev, out_ch, rows, C):
    """sv2n_head_mse_train (one launch: loss, dx, accumulated head grads) ==
    sv2n_head_mse_fwd + sv2n_head_mse_bwd with grad_loss = 1, within float
    rounding (the wave-per-rows kernel for out <= 4 sums each row's dot product
    and the gradient partials in its own fixed order); the C2 (15,360 x 50) and
    C3 (3,840 x 500) head shapes included; deterministic."""
    ops = torch.ops.sv2n
    torch.manual_seed(3)
    x = torch.randn(rows, C, device=dev)
    W = torch.randn(out_ch, C, device=dev) * 0.1
    b = torch.randn(out_ch, device=dev)
    y = torch.randn(rows * out_ch, device=dev)
    gw1, gb1 = torch.full_like(W, 0.5), torch.full_like(b, 0.25)
    gw2, gb2 = gw1.clone(), gb1.clone()
    loss1, dx1 = ops.head_mse_train(x, W, b, y, gw1, gb1)
    loss2, diff = ops.head_mse_fwd(x, W, b, y)
    dx2 = ops.head_mse_bwd(x, W, diff, torch.ones((), device=dev), gw2, gb2)
    assert_close(loss1, loss2, tol=1e-6, what="loss")
    assert_close(dx1, dx2, tol=1e-6, what="dx")
    assert_close(gw1, gw2, tol=1e-6, what="g_weight")
    assert_close(gb1, gb2, tol=1e-6, what="g_bias")
    gw3, gb3 = torch.full_like(W, 0.5), torch.full_like(b, 0.25)
    loss3, dx3 = ops.head_mse_train(x, W, b, y, gw3, gb3)
    assert torch.equal(gw1, gw3) and torch.equal(gb1, gb3)  # deterministic
    assert torch.equal(loss1, loss3) and torch.equal(dx1, dx3)


@pytest.mark.parametrize("out_ch,rows,C", [(1, 15360, 50), (3, 180, 50), (1, 3840, 500),
                                           (4, 1001, 500), (2, 777, 130), (1, 7, 500)])
def test_head_mse_train_split_is_bitwise_one_launch(dev, out_ch, rows, C):
    """sv2n_head_mse_train_rows + _reduce (ABI 19; the reduce after other
    work, as TrainStep runs it) give the one-launch sv2n_head_mse_train's loss,
    dx, accumulated head grads and loss_sum bit for bit."""
    from spotv2net_amd import library
    from spotv2net_amd.stack import head_mse_train_split
    ops = torch.ops.sv2n
    assert library.head_split_fits(C, out_ch)
    torch.manual_seed(4)
    x = torch.randn(rows, C, device=dev)
    lin = torch.nn.Linear(C, out_ch).to(dev)
    y = torch.randn(rows * out_ch, device=dev)
    with torch.no_grad():
        lin.weight.grad = torch.full_like(lin.weight, 0.5)
        lin.bias.grad = torch.full_like(lin.bias, 0.25)
    gw1, gb1 = lin.weight.grad.clone(), lin.bias.grad.clone()
    ls1 = torch.full((), 1.5, device=dev)
    ls2 = ls1.clone()
    loss1, dx1 = ops.head_mse_train(x, lin.weight.detach(), lin.bias.detach(), y, gw1, gb1, ls1)
    loss2, dx2, finish = head_mse_train_split(x, lin, y, ls2)
    _ = x * 2.0  # unrelated work between the two launches
    finish()
    torch.cuda.synchronize()
    assert torch.equal(loss1, loss2) and torch.equal(dx1, dx2)
    assert torch.equal(gw1, lin.weight.grad) and torch.equal(gb1, lin.bias.grad)
    assert torch.equal(ls1, ls2)
    # the ops themselves: shape refusal outside the wave-per-rows kernel
    assert not library.head_split_fits(2000, 1) and not library.head_split_fits(50, 5)


def test_trainstep_fused_head_matches_reference_steps(dev):
    """TrainStep's captured step (fused head+loss launch, then the GAT stack's
    backward) == k eager steps of nn.MSELoss + backward + torch.optim.Adam
    (reference 5_train_SpotV2Net.py:150-159) from the same init."""
    from spotv2net_amd import synthetic_batch
    from spotv2net_amd.train import TrainStep
    m1 = _model(dev, seed=11)
    m2 = copy.deepcopy(m1)
    data = synthetic_batch(8, 4, seed=2, device=dev)
    step = TrainStep(m1, data, lr=1e-3, use_graph=True)
    opt = torch.optim.Adam(m2.parameters(), lr=1e-3)
    for _ in range(3):
        step()
        opt.zero_grad()
        l2 = torch.nn.functional.mse_loss(m2(data), data.y_x)
        l2.backward()
        opt.step()
        assert_close(step.loss, l2.detach(), tol=1e-5, what="loss")
    for (n, p), (_, q) in zip(m1.named_parameters(), m2.named_parameters()):
        assert_close(p.detach(), q.detach(), tol=1e-5, what=n)


def test_flat_adam_advances_step_and_zeroes_grads(dev):
    from spotv2net_amd import synthetic_batch
    from spotv2net_amd.train import TrainStep
    data = synthetic_batch(8, 4, seed=6, device=dev)
    m = _model(dev, seed=4)
    s = TrainStep(m, data, use_graph=True, warmup=2)
    for _ in range(5):
        s()
    torch.cuda.synchronize()
    assert float(s.opt.step_t.item()) == 5  # replays only: the warm-up steps are undone
    assert int(s.opt.ticket.abs().sum().item()) == 0
    assert float(s.flat.abs().max().item()) == 0.0


def test_head_backward_repeatable(dev):
    """The in-launch (last-workgroup) reduction of the head's weight gradient
    leaves its ticket at zero: repeated backwards accumulate exactly."""
    from spotv2net_amd import synthetic_batch
    m = _model(dev, seed=5)
    data = synthetic_batch(40, 4, seed=7, device=dev)
    out = m(data)
    g = torch.randn_like(out)
    out.backward(g, retain_graph=True)
    first = {n: p.grad.clone() for n, p in m.named_parameters()}
    out.backward(g)
    for n, p in m.named_parameters():
        assert torch.equal(p.grad, 2 * first[n]), n


@pytest.mark.parametrize("F,H,C,nodes", [(1260, 4, 100, 15360), (70, 3, 21, 300),
                                         (300, 4, 48, 3000), (40, 3, 5, 120), (16, 2, 1, 60)])
def test_fused_wgrad_matches_gemm_and_fold(dev, F, H, C, nodes):
    """sv2n_gat_wgrad_node (split-K GEMM + fused epilogue) against the
    unfused sv2n_gemm_f32 + sv2n_gat_prep_bwd_node path it replaces; two
    accumulating calls, then a bias-only call.  Shapes: the C2 layer 0
    (k_gemm_tt3y, 208-column tiles), a ragged one on the same kernel (F 300:
    a partial row block; 200 columns), one on the f32 kernel, and narrow heads
    (C 5, C 1)."""
    from spotv2net_amd import _lib
    from spotv2net_amd.ops import gemm_f32
    lib = _lib.load()
    g = torch.Generator(device="cpu").manual_seed(11)
    HC = H * C
    ldx = (HC + 2 * H + 3) // 4 * 4
    x = torch.randn(nodes, F, generator=g).to(dev)
    dxs = torch.randn(nodes, ldx, generator=g).to(dev)
    W = torch.randn(HC, F, generator=g).to(dev)
    a_s = torch.randn(H, C, generator=g).to(dev)
    a_d = torch.randn(H, C, generator=g).to(dev)
    B = max(1, nodes // 30)
    dbp = torch.randn(B, HC, generator=g).to(dev)
    st = _lib.stream_handle(dev)

    def grads():
        return [torch.zeros(HC, F, device=dev), torch.zeros(H, C, device=dev),
                torch.zeros(H, C, device=dev), torch.zeros(HC, device=dev)]

    ref = grads()
    T = gemm_f32(x, False, dxs, False, F, ldx, nodes)
    ws_n = lib.sv2n_gat_prep_bwd_workspace(H, F)
    wsr = torch.empty(ws_n, device=dev)
    _lib.check(lib.sv2n_gat_prep_bwd_node(T.data_ptr(), ldx, W.data_ptr(), a_s.data_ptr(),
                                          a_d.data_ptr(), H, C, F, dbp.data_ptr(), B, HC,
                                          *[r.data_ptr() for r in ref], wsr.data_ptr(), ws_n, st),
               "prep_bwd_node")
    got = grads()
    ws_n = lib.sv2n_gat_wgrad_node_workspace(nodes, F, ldx, H, C)
    ws = torch.zeros(ws_n, device=dev)
    for _ in range(2):
        _lib.check(lib.sv2n_gat_wgrad_node(x.data_ptr(), x.stride(0), dxs.data_ptr(), ldx, nodes,
                                           F, W.data_ptr(), a_s.data_ptr(), a_d.data_ptr(), H, C,
                                           dbp.data_ptr(), B, HC, *[r.data_ptr() for r in got],
                                           ws.data_ptr(), ws_n, st), "wgrad_node")
    torch.cuda.synchronize()
    for r, o, name in zip(ref, got, ("gW", "g_att_src", "g_att_dst", "g_bias")):
        assert_close(o, 2 * r, tol=2e-5, what=name)
    gb = torch.zeros(HC, device=dev)
    _lib.check(lib.sv2n_gat_wgrad_node(None, 0, None, ldx, nodes, F, None, None, None, H, C,
                                       dbp.data_ptr(), B, HC, None, None, None, gb.data_ptr(),
                                       ws.data_ptr(), ws_n, st), "wgrad bias only")
    assert_close(gb, ref[3], tol=1e-6, what="bias only")


def test_trainstep_standardize_matches_reference_steps(dev):
    """standardize=True (BatchNorm over x and edge_attr, utils/models.py:76-78,
    :141-143; the yaml grid's option, GNN_param.yaml:70): the captured step's
    warm-up is undone for the running statistics too, so k TrainStep calls ==
    k eager reference steps — parameters AND buffers."""
    from spotv2net_amd import synthetic_batch
    from spotv2net_amd.train import TrainStep
    m1 = _model(dev, seed=12, standardize=True)
    m2 = copy.deepcopy(m1)
    data = synthetic_batch(8, 4, seed=3, device=dev)
    step = TrainStep(m1, data, lr=1e-3, use_graph=True, warmup=3)
    for (n, b), (_, c) in zip(m1.named_buffers(), m2.named_buffers()):
        assert torch.equal(b, c), f"{n}: constructing a TrainStep must not move the buffers"
    opt = torch.optim.Adam(m2.parameters(), lr=1e-3)
    for _ in range(3):
        step()
        opt.zero_grad()
        l2 = torch.nn.functional.mse_loss(m2(data), data.y_x)
        l2.backward()
        opt.step()
        assert_close(step.loss, l2.detach(), tol=1e-5, what="loss")
    for (n, p), (_, q) in zip(m1.named_parameters(), m2.named_parameters()):
        assert_close(p.detach(), q.detach(), tol=1e-5, what=n)
    for (n, b), (_, c) in zip(m1.named_buffers(), m2.named_buffers()):
        if b.dtype == torch.long:
            assert torch.equal(b, c), n
        else:
            assert_close(b, c, tol=1e-6, what=n)
