"""sv2n_gemm_f32 (f32 MFMA) against float64 torch for all operand layouts,
ragged sizes and the split-K path."""
import pytest
import torch

from helpers import assert_close

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("a_k,b_k", [(True, True), (True, False), (False, False), (False, True)])
@pytest.mark.parametrize("M,N,K", [(15360 // 8, 408, 1260), (333, 77, 5), (64, 208, 16),
                                   (1260, 408, 15360 // 4), (130, 129, 131), (1, 1, 1)])
def test_gemm_layouts(dev, a_k, b_k, M, N, K):
    from spotv2net_amd.ops import gemm_f32
    torch.manual_seed(M + N + K)
    A = torch.randn(M, K, device=dev)
    B = torch.randn(N, K, device=dev)
    a_arg = A if a_k else A.t().contiguous()
    b_arg = B if b_k else B.t().contiguous()
    C = gemm_f32(a_arg, a_k, b_arg, b_k, M, N, K)
    ref = A.double() @ B.double().t()
    # f32 accumulation over K terms of |a b| ~ 1: allow sqrt(K)-scaled rounding
    tol = 1e-5 * max(1.0, (K ** 0.5) / 8)
    assert_close(C, ref, tol=tol, what="gemm")


def test_linear_autograd(dev):
    from spotv2net_amd.ops import linear
    torch.manual_seed(0)
    x = torch.randn(600, 90, device=dev, requires_grad=True)
    w = torch.randn(52, 90, device=dev, requires_grad=True)
    y = linear(x, w)
    g = torch.randn_like(y)
    y.backward(g)
    xr = x.detach().double().requires_grad_(True)
    wr = w.detach().double().requires_grad_(True)
    (xr @ wr.t()).backward(g.double())
    assert_close(y, xr @ wr.t(), what="y")
    assert_close(x.grad, xr.grad, what="dx")
    assert_close(w.grad, wr.grad, what="dw")


@pytest.mark.parametrize("M,N,K,transpose", [(15360, 408, 1260, False), (300, 17, 5, False),
                                             (257, 400, 208, True), (64, 1, 70, True),
                                             (1000, 130, 64, False), (15360, 400, 208, False),
                                             (15360, 208, 400, False), (4000, 208, 1260, True),
                                             (100, 50, 4, False), (129, 208, 36, False),
                                             (300, 144, 1024, False)])
def test_split3_gemm_matches_f32_accuracy(dev, M, N, K, transpose):
    """sv2n_gemm_f32x3 (three bf16 planes, six MFMA products) is as close to
    the float64 product as the exact-f32 MFMA GEMM: max error relative to
    Σ|a·b| within 2x of sv2n_gemm_f32's, and below 1e-6."""
    from spotv2net_amd import ops
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    a = torch.randn(M, K, generator=g).to(dev)
    w = (torch.randn(K, N, generator=g) if transpose else torch.randn(N, K, generator=g)).to(dev)
    w = w.contiguous()
    got = ops.project(a, w, transpose)
    wb = w if transpose else w.t()                      # [K][N]
    ref = (a.double() @ wb.double())
    scale = (a.double().abs() @ wb.double().abs())
    f32 = ops.gemm_f32(a, True, w, not transpose, M, N, K)
    e3 = ((got.double() - ref).abs() / scale.clamp_min(1e-30)).max().item()
    e32 = ((f32.double() - ref).abs() / scale.clamp_min(1e-30)).max().item()
    assert e3 < 1e-6 and e3 <= 2 * e32 + 1e-9, (e3, e32)


@pytest.mark.parametrize("M,N,K", [(15360, 400, 208), (15360, 208, 400), (300, 144, 1024),
                                   (129, 50, 36)])
def test_split3_gemm_relu_mask_is_exact(dev, M, N, K):
    """sv2n_gemm_f32x3_relu stores (y > 0) ? A·Bᵀ : 0: bit-identical to the
    unmasked GEMM where y > 0, exact zeros elsewhere (ReLU's backward, as the
    n <= 32 attention backward applies it: act_bwd<ACT_RELU>); y with exact
    zeros, positives and negatives, and a row stride wider than N."""
    from spotv2net_amd import _lib, ops
    lib = _lib.load()
    g = torch.Generator(device="cpu").manual_seed(M + 7 * N + K)
    a = torch.randn(M, K, generator=g).to(dev)
    w = torch.randn(K, N, generator=g).to(dev)
    planes = ops.weight_planes(w, True)
    plain = ops.project_planes(a, planes, w, True)
    yb = torch.randn(M, N + 8, generator=g)
    yb[yb.abs() < 0.3] = 0.0
    y = yb.to(dev)[:, :N]
    got = ops.project_planes(a, planes, w, True, relu_y=y)
    assert torch.equal(got, torch.where(y > 0, plain, torch.zeros_like(plain)))
    out = torch.empty_like(plain)
    st = _lib.stream_handle(dev)
    # K % 4 != 0 is refused before any launch (the caller masks in the attention)
    assert lib.sv2n_gemm_f32x3_relu(a.data_ptr(), K, planes.data_ptr(), out.data_ptr(), N, M, N,
                                    K - 1, y.data_ptr(), y.stride(0), st) == -2
    assert lib.sv2n_gemm_f32x3_relu(a.data_ptr(), K, planes.data_ptr(), out.data_ptr(), N, M, N,
                                    K, None, 0, st) == -1


def test_prep_fwd_all_matches_per_layer(dev):
    """sv2n_gat_prep_fwd_all (one launch, all layers) equals sv2n_gat_prep_fwd
    + sv2n_split3 (+ the transposed split) per layer, bit for bit."""
    import ctypes
    from spotv2net_amd import _lib
    lib = _lib.load()
    st = _lib.stream_handle(dev)
    g = torch.Generator().manual_seed(3)
    shapes = [(4, 100, 1260), (4, 50, 400)]  # (H, C, F) of the C2 layers
    D, H = 126, 4
    hp = 8
    arr = (_lib.PrepLayer * len(shapes))()
    keep = []
    wf_all = torch.zeros(D, hp, device=dev)
    wf_ref = torch.zeros(D, hp, device=dev)
    for l, (Hh, C, F) in enumerate(shapes):
        HC = Hh * C
        ldx = (HC + 2 * Hh + 3) // 4 * 4
        W = torch.randn(HC, F, generator=g).to(dev)
        a_s, a_d, a_e = (torch.randn(HC, generator=g).to(dev) for _ in range(3))
        We = torch.randn(HC, D, generator=g).to(dev)
        kp, kpt = lib.sv2n_split3_kpad(F), lib.sv2n_split3_kpad(ldx)
        waug = torch.empty(ldx, F, device=dev)
        pl = torch.empty(3, ldx, kp, device=dev, dtype=torch.int16)
        plt = torch.empty(3, F, kpt, device=dev, dtype=torch.int16)
        arr[l] = _lib.PrepLayer(W.data_ptr(), a_s.data_ptr(), a_d.data_ptr(), Hh, C, F, ldx,
                                waug.data_ptr(), pl.data_ptr(), plt.data_ptr(), We.data_ptr(),
                                a_e.data_ptr(), D, hp, l * H, wf_all.data_ptr())
        # reference: the per-layer entries
        waug_r = torch.empty(ldx, F, device=dev)
        _lib.check(lib.sv2n_gat_prep_fwd(W.data_ptr(), a_s.data_ptr(), a_d.data_ptr(), Hh, C, F,
                                         waug_r.data_ptr(), ldx, We.data_ptr(), a_e.data_ptr(), D,
                                         wf_ref.data_ptr(), hp, l * H, st), "prep_fwd")
        pl_r = torch.empty(3, ldx, kp, device=dev, dtype=torch.int16)
        _lib.check(lib.sv2n_split3(waug_r.data_ptr(), ldx, F, F, 0, pl_r.data_ptr(), st), "split3")
        plt_r = torch.empty(3, F, kpt, device=dev, dtype=torch.int16)
        _lib.check(lib.sv2n_split3(waug_r.data_ptr(), F, ldx, F, 1, plt_r.data_ptr(), st),
                   "split3 transposed")
        keep.append((W, a_s, a_d, a_e, We, waug, pl, plt, waug_r, pl_r, plt_r))
    _lib.check(lib.sv2n_gat_prep_fwd_all(ctypes.addressof(arr), len(shapes), st), "prep_fwd_all")
    torch.cuda.synchronize()
    for (*_, waug, pl, plt, waug_r, pl_r, plt_r) in keep:
        assert torch.equal(waug, waug_r)
        assert torch.equal(pl, pl_r)
        assert torch.equal(plt, plt_r)
    assert torch.equal(wf_all, wf_ref)


def test_prep_fwd_all_without_waug(dev):
    """ABI 19: sv2n_gat_prep_fwd_all with waug NULL (bf16 mode) writes the same
    planes (and planes_t, wfold) as with waug, and nothing in place of waug."""
    import ctypes
    from spotv2net_amd import _lib
    lib = _lib.load()
    st = _lib.stream_handle(dev)
    g = torch.Generator().manual_seed(4)
    shapes = [(6, 500, 1260), (6, 30, 3012)]  # C3-sized layer 0, a second layer
    D, H, hp = 126, 6, 12
    runs = []
    for with_waug in (True, False):
        arr = (_lib.PrepLayer * len(shapes))()
        wf = torch.zeros(D, hp, device=dev)
        keep = []
        for l, (Hh, C, F) in enumerate(shapes):
            g.manual_seed(10 + l)
            HC = Hh * C
            ldx = (HC + 2 * Hh + 3) // 4 * 4
            W = torch.randn(HC, F, generator=g).to(dev)
            a_s, a_d, a_e = (torch.randn(HC, generator=g).to(dev) for _ in range(3))
            We = torch.randn(HC, D, generator=g).to(dev)
            kp, kpt = lib.sv2n_split3_kpad(F), lib.sv2n_split3_kpad(ldx)
            waug = torch.full((ldx, F), 7.0, device=dev)
            pl = torch.empty(1, ldx, kp, device=dev, dtype=torch.int16)
            plt = torch.empty(1, F, kpt, device=dev, dtype=torch.int16)
            arr[l] = _lib.PrepLayer(W.data_ptr(), a_s.data_ptr(), a_d.data_ptr(), Hh, C, F, ldx,
                                    waug.data_ptr() if with_waug else None, pl.data_ptr(),
                                    plt.data_ptr(), We.data_ptr(), a_e.data_ptr(), D, hp, l * H,
                                    wf.data_ptr(), 1)
            keep.append((W, a_s, a_d, a_e, We, waug, pl, plt))
        _lib.check(lib.sv2n_gat_prep_fwd_all(ctypes.addressof(arr), len(shapes), st),
                   "prep_fwd_all")
        torch.cuda.synchronize()
        runs.append((keep, wf))
    (with_k, wf_a), (without_k, wf_b) = runs
    assert torch.equal(wf_a, wf_b)
    for a, b in zip(with_k, without_k):
        assert torch.equal(a[6], b[6]) and torch.equal(a[7], b[7])
        assert not torch.equal(a[5], b[5])  # written with, untouched without
        assert bool((b[5] == 7.0).all())


def test_bf16_prep_waug_placeholder(dev):
    """bf16-mode gat_prep returns Waug as a stride-0 placeholder of its shape;
    the projections that take the planes run, the ones that would read Waug
    refuse it loudly."""
    from spotv2net_amd import GATModel, library  # noqa: F401
    ops = torch.ops.sv2n
    torch.manual_seed(0)
    m = GATModel(60, 6, 2, 1, [8, 4], concat_heads=True).to(dev)
    c0, c1 = m.gat_layers
    args = ([c0.lin_src.weight, c1.lin_src.weight], [c0.att_src, c1.att_src],
            [c0.att_dst, c1.att_dst], [c0.lin_edge.weight, c1.lin_edge.weight],
            [c0.att_edge, c1.att_edge], [2, 2], [8, 4], 4, [False, True], True)
    w32, p32, _, wf32 = ops.gat_prep(*args, bf16=False)
    w16, p16, pt16, wf16 = ops.gat_prep(*args, bf16=True)
    assert torch.equal(wf32, wf16)
    for a, b, pl in zip(w32, w16, p16):
        assert b.shape == a.shape and b.stride() == (0, 0)
        # plane 0 of bf16 mode is bf16_rn(Waug) (zero past F)
        ref = a.to(torch.bfloat16).view(torch.int16)
        assert torch.equal(pl[0, :, :a.shape[1]], ref)
    x = torch.randn(96, 60, device=dev)
    xs = ops.project(x, p16[0], w16[0], False, True)
    assert xs.shape == (96, w32[0].shape[0])
    with pytest.raises(RuntimeError, match="placeholder"):
        ops.project(x, None, w16[0], False, True)
    with pytest.raises(RuntimeError, match="placeholder"):
        ops.project(x, None, w16[0], False, False)
