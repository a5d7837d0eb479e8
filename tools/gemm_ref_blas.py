"""Time hipBLASLt/rocBLAS (torch.matmul, fp32) on the C2 projection GEMM
shapes: the known-good reference point for sv2n_gemm_f32 on the same GPU."""
import torch

shapes = [("fwd L0", 15360, 408, 1260, True, True), ("fwd L1", 15360, 208, 400, True, True),
          ("dX  L1", 15360, 400, 208, True, False), ("dWT L0", 1260, 408, 15360, False, False),
          ("dWT L1", 400, 208, 15360, False, False)]
torch.backends.cuda.matmul.allow_tf32 = False
dev = torch.device("cuda")
for name, M, N, K, ak, bk in shapes:
    A = torch.rand(M, K, device=dev) * 2 - 1
    B = torch.rand(N, K, device=dev) * 2 - 1
    a = A if ak else A.t().contiguous().t()   # logical [M,K] with the tuned memory layout
    b = (B if bk else B.t().contiguous().t()).t()
    for _ in range(5):
        c = a @ b
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        c = a @ b
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 20
    print(f"{name} M={M} N={N} K={K}: torch.matmul {us:8.1f} us {2*M*N*K/us/1e6:6.1f} TF")
