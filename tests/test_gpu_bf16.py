"""bf16 execution mode (BASELINE config C3: the reference under bf16
autocast) and the wide output head (C1 / C3 hidden 500).

Kernel-level checks are exact-arithmetic ones: sv2n_gemm_bf16 and the bf16
weight-gradient GEMM must equal float64 products of the bf16-ROUNDED operands
to fp32 accumulation error.  Model-level checks compare the bf16 mode with
the fp32 oracle at a bf16 tolerance (BF16_TOL, scaled like helpers.TOL)."""
import pytest
import torch

from helpers import assert_close, twin_model

pytestmark = pytest.mark.gpu

BF16_TOL = 2e-2  # bf16 operands carry 8 significant bits (2^-9 relative rounding)


def _bf(t):
    return t.to(torch.bfloat16).to(torch.float32)


def _rel_to_abs_sum(got, a, b):
    """max |got - a·bᵀ| / max Σ_k |a_k b_k| over the output (float64 truth)."""
    ref = a.double() @ b.double().t()
    absum = a.double().abs() @ b.double().abs().t()
    return ((got.double() - ref).abs() / absum.clamp_min(1e-30)).max().item()


@pytest.mark.parametrize("M,N,K", [(3840, 3012, 1260), (15360, 408, 1260), (97, 37, 72),
                                   (1100, 389, 332)])
def test_gemm_bf16_is_exact_bf16_products(dev, M, N, K):
    from spotv2net_amd import _lib
    from spotv2net_amd.ops import weight_planes
    lib = _lib.load()
    g = torch.Generator().manual_seed(M + N)
    a = torch.randn(M, K, generator=g).to(dev)
    w = (torch.randn(N, K, generator=g) * 0.05).to(dev)
    planes = weight_planes(w, False)
    out = torch.empty(M, N, device=dev)
    _lib.check(lib.sv2n_gemm_bf16(a.data_ptr(), a.stride(0), planes.data_ptr(), out.data_ptr(),
                                  N, M, N, K, _lib.stream_handle(dev)), "gemm_bf16")
    err = _rel_to_abs_sum(out.cpu(), _bf(a).cpu(), _bf(w).cpu())
    assert err < 2e-6, err  # fp32 accumulation of exact bf16 x bf16 products


def test_project_planes_bf16_unaligned_rows(dev):
    """The bf16 projection on activations whose row length is not a multiple of
    4 floats (e.g. a 50-wide layer input): padded to 16-B rows, same products."""
    from spotv2net_amd.ops import project_planes
    g = torch.Generator().manual_seed(5)
    a = torch.randn(300, 70, generator=g).to(dev)
    w = (torch.randn(37, 70, generator=g) * 0.1).to(dev)
    out = project_planes(a, None, w, False, bf16=True)
    err = _rel_to_abs_sum(out.cpu(), _bf(a).cpu(), _bf(w).cpu())
    assert err < 2e-6, err


@pytest.mark.parametrize("F,H,C,nodes", [(1260, 6, 500, 3840), (1260, 4, 100, 15360),
                                         (72, 3, 21, 300), (70, 3, 21, 300), (332, 5, 77, 1010)])
def test_wgrad_bf16_equals_f32_on_rounded_operands(dev, F, H, C, nodes):
    """sv2n_gat_wgrad_node_bf16 == sv2n_gat_wgrad_node (exact f32) fed the
    bf16-rounded x and dxs: the bf16 GEMM's products are exact, so only the
    summation order differs.  F % 4 == 0 runs the transposed product with the
    slab-summing epilogue (k_wgrad_epi_t); F = 70 (x rows padded to 72) the
    [F][ldx] product, the reduce launch and k_wgrad_epi."""
    from spotv2net_amd import _lib
    lib = _lib.load()
    g = torch.Generator().manual_seed(F + C)
    HC = H * C
    ldx = (HC + 2 * H + 3) // 4 * 4
    ldin = (F + 3) // 4 * 4
    x = torch.zeros(nodes, ldin)
    x[:, :F] = torch.randn(nodes, F, generator=g)
    x = x.to(dev)
    dxs = (torch.randn(nodes, ldx, generator=g) * 1e-3).to(dev)
    W = (torch.randn(HC, F, generator=g) * 0.03).to(dev)
    a_s = torch.randn(H, C, generator=g).to(dev)
    a_d = torch.randn(H, C, generator=g).to(dev)
    B = max(1, nodes // 30)
    dbp = torch.randn(B, HC, generator=g).to(dev)
    st = _lib.stream_handle(dev)

    def run(fn, wsfn, xx, dd):
        outs = [torch.zeros(HC, F, device=dev), torch.zeros(H, C, device=dev),
                torch.zeros(H, C, device=dev), torch.zeros(HC, device=dev)]
        n = wsfn(nodes, F, ldx, H, C)
        ws = torch.zeros(n, device=dev)
        _lib.check(fn(xx.data_ptr(), ldin, dd.data_ptr(), ldx, nodes, F, W.data_ptr(),
                      a_s.data_ptr(), a_d.data_ptr(), H, C, dbp.data_ptr(), B, HC,
                      *[o.data_ptr() for o in outs], ws.data_ptr(), n, st), "wgrad")
        return outs

    got = run(lib.sv2n_gat_wgrad_node_bf16, lib.sv2n_gat_wgrad_node_bf16_workspace, x, dxs)
    ref = run(lib.sv2n_gat_wgrad_node, lib.sv2n_gat_wgrad_node_workspace, _bf(x), _bf(dxs))
    for o, r, name in zip(got, ref, ("gW", "g_att_src", "g_att_dst", "g_bias")):
        scale = max(r.abs().max().item(), 1e-30)
        e = (o - r).abs().max().item() / scale
        assert e < 2e-5, f"{name}: {e:.3e}"


@pytest.mark.parametrize("C,O", [(500, 1), (500, 14), (200, 3), (129, 16)])
def test_wide_head_kernels(dev, C, O):
    """sv2n_head_* for in_features > 128 (C1/C3 hidden 500): forward, fused
    MSE, and backward against float64."""
    from spotv2net_amd.stack import head_fits, head_mse_loss, linear_head
    assert head_fits(C, O)
    torch.manual_seed(C + O)
    lin = torch.nn.Linear(C, O).to(dev)
    x = torch.randn(3000, C, device=dev, requires_grad=True)
    y = torch.randn(3000 * O, device=dev)
    xr = x.detach().cpu().double().requires_grad_(True)
    wr = lin.weight.detach().cpu().double().requires_grad_(True)
    br = lin.bias.detach().cpu().double().requires_grad_(True)
    out = linear_head(x, lin)
    ref = torch.nn.functional.linear(xr, wr, br)
    assert_close(out, ref, what="head fwd")
    loss = head_mse_loss(x, lin, y)
    rloss = torch.nn.functional.mse_loss(ref.view(-1), y.cpu().double())
    assert_close(loss, rloss, what="loss")
    loss.backward()
    rloss.backward()
    assert_close(x.grad, xr.grad, what="dx")
    assert_close(lin.weight.grad, wr.grad, what="dW")
    assert_close(lin.bias.grad, br.grad, what="db")


def test_c3_model_bf16_close_to_fp32_oracle(dev):
    """The yaml C3 model in bf16 mode against the fp32 oracle: forward and
    every gradient within BF16_TOL (scaled by max(1, |ref|))."""
    from spotv2net_amd import Data, synthetic_batch
    S = 42
    mine, ref = twin_model(seed=5154, num_node_features=30 * S, num_edge_features=3 * S,
                           num_heads=6, output_node_channels=1, dim_hidden_layers=[500],
                           concat_heads=True)
    mine = mine.to(dev).set_precision("bf16")
    data = synthetic_batch(16, S, seed=21)
    gd = data.to(dev)
    out = mine(gd)
    torch.nn.functional.mse_loss(out, gd.y_x).backward()
    rout = ref(Data(x=data.x, edge_index=data.edge_index, edge_attr=data.edge_attr))
    torch.nn.functional.mse_loss(rout, data.y_x).backward()
    assert_close(out, rout, tol=BF16_TOL, what="forward")
    for (name, p), (_, q) in zip(mine.named_parameters(), ref.named_parameters()):
        assert_close(p.grad, q.grad, tol=BF16_TOL, what=f"d{name}")


@pytest.mark.parametrize("x_grad", [False, True])
def test_bf16_eval_mode_backward(dev, x_grad):
    """model.eval() and still a backward (a gradient asked for outside
    training): the bf16 mode's dX GEMMs need the transposed weight planes,
    since its f32 Waug is a placeholder.  Two layers, so layer 1's dX runs;
    with x.requires_grad layer 0's too.  Against the fp32 oracle at BF16_TOL."""
    from spotv2net_amd import Data, synthetic_batch
    S = 4
    mine, ref = twin_model(seed=11, num_node_features=30 * S, num_edge_features=3 * S,
                           num_heads=4, output_node_channels=1, dim_hidden_layers=[24, 12],
                           concat_heads=True)
    mine = mine.to(dev).set_precision("bf16").eval()
    ref.eval()
    data = synthetic_batch(6, S, seed=4)
    x = data.x.clone().to(dev).requires_grad_(x_grad)
    gd = Data(x=x, edge_index=data.edge_index.to(dev), edge_attr=data.edge_attr.to(dev))
    out = mine(gd)
    torch.nn.functional.mse_loss(out, data.y_x.to(dev)).backward()
    xr = data.x.clone().requires_grad_(x_grad)
    rout = ref(Data(x=xr, edge_index=data.edge_index, edge_attr=data.edge_attr))
    torch.nn.functional.mse_loss(rout, data.y_x).backward()
    assert_close(out, rout, tol=BF16_TOL, what="forward")
    for (name, p), (_, q) in zip(mine.named_parameters(), ref.named_parameters()):
        assert_close(p.grad, q.grad, tol=BF16_TOL, what=f"d{name}")
    if x_grad:
        assert_close(x.grad, xr.grad, tol=BF16_TOL, what="dx")


def test_autocast_selects_bf16_mode(dev):
    """Inside torch.autocast("cuda", dtype=torch.bfloat16) the model runs the
    bf16 mode (as set_precision("bf16")); outside it, fp32."""
    from spotv2net_amd import GATModel, synthetic_batch
    torch.manual_seed(3)
    m = GATModel(30 * 4, 3 * 4, 4, 1, [16, 8], concat_heads=True).to(dev)
    data = synthetic_batch(4, 4, seed=3, device=dev)
    with torch.no_grad():
        f32 = m(data)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            auto = m(data)
        m.set_precision("bf16")
        forced = m(data)
    assert auto.dtype == torch.float32
    assert torch.equal(auto, forced)
    assert not torch.equal(auto, f32)
    assert (auto - f32).abs().max().item() < 5e-2
