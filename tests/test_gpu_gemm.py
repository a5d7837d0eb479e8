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
