"""bf16 execution mode (BASELINE C3: the reference under bf16 autocast) with
the weight-gradient operands kept in bf16 (ABI 14): layer 0's projection
exports bf16(x) (sv2n_gemm_bf16_export), its attention backward writes dxs as
bf16 (sv2n_gat_attn_bwd_bf16dx) and the weight-gradient GEMM reads both
(sv2n_gat_wgrad_node_bf16b).  The roundings are the ones the fp32-operand
GEMMs apply while staging, so the operands are bit-identical to the fp32
path's and the gradients differ only by the split-K summation order."""
import copy

import pytest
import torch

from helpers import assert_close

pytestmark = pytest.mark.gpu


def test_projection_export_is_bf16_of_x(dev):
    from spotv2net_amd import ops
    torch.manual_seed(0)
    for M, K, N in ((3840, 1260, 3012), (200, 60, 40)):   # large-tile path; the rounding pass
        x = torch.randn(M, K, device=dev)
        w = torch.randn(N, K, device=dev) * 0.05
        planes = ops.weight_planes(w, False)
        out, xb = torch.ops.sv2n.project_bf16_export(x, planes, w)
        ref = torch.ops.sv2n.project(x, planes, w, False, True)
        assert torch.equal(out, ref)
        assert xb.shape[1] % 64 == 0 and xb.shape[1] >= K
        assert torch.equal(xb[:, :K], x.to(torch.bfloat16))
        assert not xb[:, K:].float().abs().any()


@pytest.mark.parametrize("concat,post", [(False, 0.0), (True, 0.1)])
def test_attention_backward_bf16_dxs_is_rounded_fp32(dev, concat, post):
    from spotv2net_amd import synthetic_batch
    from spotv2net_amd.model import _layout_of
    B, S, H, C = 24, 2, 3, 20
    data = synthetic_batch(B, S, seed=3, device=dev)
    layout = _layout_of(data, data.x, data.edge_index)
    N = B * 30
    torch.manual_seed(1)
    ldx = (H * C + 2 * H + 3) // 4 * 4
    xs = torch.randn(N, ldx, device=dev)
    ae = torch.randn(B * 870, H, device=dev)
    OC = H * C if concat else C
    bias = torch.randn(OC, device=dev)
    u = torch.rand(N, OC, device=dev) if post else None
    if post:
        y, ps, _ = torch.ops.sv2n.gat_attn_fwd_post(xs, ae, None, bias, None, 1.0, u, post, B, 30,
                                                   H, C, concat, 1, 0.2, True)
    else:
        y, ps = torch.ops.sv2n.gat_attn_fwd(xs, ae, None, bias, None, 1.0, B, 30, H, C, concat,
                                            1, 0.2, True)
    dy = torch.randn(N, OC, device=dev)
    dxs, dae, dbp = torch.ops.sv2n.gat_attn_bwd(dy, y, xs, ps, None, 1.0, layout.rowmask, True,
                                                B, 30, H, C, concat, 1, 0.2, True, u, post)
    dxb, dae2, dbp2 = torch.ops.sv2n.gat_attn_bwd_bf16dx(dy, y, xs, ps, None, 1.0,
                                                         layout.rowmask, True, B, 30, H, C,
                                                         concat, 1, 0.2, True, u, post)
    assert torch.equal(dxb[:, :ldx], dxs.to(torch.bfloat16))
    assert not dxb[:, ldx:].float().abs().any()
    assert torch.equal(dae, dae2) and torch.equal(dbp, dbp2)


@pytest.mark.parametrize("S,heads,hidden,B,dropout", [
    (2, 6, [40], 16, 0.1),        # C3's structure (one mean layer, post-layer dropout)
    (2, 4, [16, 8], 12, 0.0),     # two layers: layer 1's dxs stays fp32 (it feeds dX)
])
def test_bf16_operand_path_matches_fp32_operands(dev, S, heads, hidden, B, dropout):
    from spotv2net_amd import GATModel, stack, synthetic_batch
    torch.manual_seed(4)
    m1 = GATModel(30 * S, 3 * S, heads, 1, hidden, concat_heads=True, dropout=dropout).to(dev)
    m1.set_precision("bf16")
    m1.graph_replay = False
    m2 = copy.deepcopy(m1)
    data = synthetic_batch(B, S, seed=8, device=dev)
    grads = []
    for m, mode in ((m1, "on"), (m2, "off")):
        old = stack.BF16_OPERANDS
        stack.BF16_OPERANDS = mode
        try:
            torch.cuda.manual_seed(5)
            loss = torch.nn.functional.mse_loss(m(data), data.y_x)
            loss.backward()
            torch.cuda.synchronize()
        finally:
            stack.BF16_OPERANDS = old
        grads.append({n: p.grad.detach().clone() for n, p in m.named_parameters()})
    for name in grads[0]:
        assert_close(grads[0][name], grads[1][name], tol=2e-6, what=name)


@pytest.mark.parametrize("n,S,Fs", [(30, 42, 1), (30, 4, 14)])
def test_window_gather_bf16_twin(dev, n, S, Fs):
    """WindowDataset.empty_batch(bf16_x=True): the gather writes bf16(x)
    beside x (sv2n_window_gather_bf16x, ABI 15) — bit for bit x rounded to
    nearest even, zero past n·S, NaN rows for windows outside the series —
    and x, edge_attr, y_x as without it."""
    from spotv2net_amd import WindowDataset
    from spotv2net_amd.data import bf16_twin, synthetic_series
    V, W = synthetic_series(S + Fs + 60, n, seed=n + S)
    ds = WindowDataset(V.to(dev), W.to(dev), S, cut=3, future_steps=Fs)
    idx = torch.randperm(len(ds), generator=torch.Generator().manual_seed(2))[:33].to(dev)
    idx[5] = 10 ** 6   # past the series: NaN rows
    a = ds.empty_batch(idx.numel(), bf16_x=True)
    b = ds.empty_batch(idx.numel())
    ds.fill(a, idx)
    ds.fill(b, idx)
    xb = bf16_twin(a)
    assert xb is not None and bf16_twin(b) is None
    for key in ("x", "edge_attr", "y_x"):
        assert torch.equal(getattr(a, key).nan_to_num(7.0), getattr(b, key).nan_to_num(7.0)), key
    K = n * S
    assert torch.equal(xb[:, :K].float().nan_to_num(7.0), a.x.to(torch.bfloat16).float().nan_to_num(7.0))
    assert not xb[:, K:].float().abs().any()
    a.x.add_(0.0)   # an in-place write to x retires the twin
    assert bf16_twin(a) is None


def test_bf16_twin_step_is_bit_identical(dev):
    """The C3 model in bf16 mode on a WindowDataset batch with and without the
    bf16 twin of x: the same roundings feed the same GEMMs, so the output and
    every gradient are bit-identical (project_a16 vs the exporting projection)."""
    from spotv2net_amd import GATModel, WindowDataset
    from spotv2net_amd.data import synthetic_series
    S = 42
    V, W = synthetic_series(S + 200, 30, seed=3)
    ds = WindowDataset(V.to(dev), W.to(dev), S, cut=5)
    idx = torch.arange(40, device=dev)
    a, b = ds.empty_batch(40, bf16_x=True), ds.empty_batch(40)
    ds.fill(a, idx)
    ds.fill(b, idx)
    torch.manual_seed(4)
    m1 = GATModel(30 * S, 3 * S, 6, 1, [500], concat_heads=True).to(dev).set_precision("bf16")
    m1.graph_replay = False
    m2 = copy.deepcopy(m1)
    outs = []
    for m, d in ((m1, a), (m2, b)):
        out = m(d)
        torch.nn.functional.mse_loss(out, d.y_x).backward()
        outs.append(out.detach())
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    for (n1, p), (_, q) in zip(m1.named_parameters(), m2.named_parameters()):
        assert torch.equal(p.grad, q.grad), n1
