"""What the vendor library reaches on the C3 GEMM shapes (bf16 operands):
torch.matmul (hipBLASLt) for the projection x·Waugᵀ (3840 x 3012 x 1260) and
the weight gradient xᵀ·dxs (1260 x 3012 x 3840), both operand layouts as they
lie in memory.  A yardstick for k_gemm_bf16nt / k_gemm_tt, not a product path."""
import torch


def t(fn, reps=50):
    for _ in range(5):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


dev = torch.device("cuda", 0)
x = torch.randn(3840, 1260, device=dev, dtype=torch.bfloat16)
w = torch.randn(3012, 1260, device=dev, dtype=torch.bfloat16)
d = torch.randn(3840, 3012, device=dev, dtype=torch.bfloat16)
fl = 2 * 3840 * 3012 * 1260
for name, fn in [("proj x.wT", lambda: x @ w.t()), ("wgrad xT.d", lambda: x.t() @ d),
                 ("proj f32out", lambda: torch.matmul(x, w.t()).float())]:
    us = t(fn)
    print(f"{name:14s} {us:7.1f} us {fl / us / 1e6:7.1f} TF/s", flush=True)
