"""Time the n <= 32 attention kernels (HIP events on the launch stream) on the
C2 / C3 layer shapes; run under different SV2N_ATT_TARGET_WG values."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spotv2net_amd import library  # noqa: F401,E402

ops = torch.ops.sv2n
dev = torch.device("cuda")


def bench(fn, reps=50):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


for name, B, H, C, concat in [("C2 L0", 512, 4, 100, True), ("C2 L1", 512, 4, 50, False),
                              ("C3", 128, 6, 500, False)]:
    n = 30
    ldx = (H * C + 2 * H + 3) // 4 * 4
    xs = torch.randn(B * n, ldx, device=dev)
    ae = torch.randn(B * n * (n - 1), H, device=dev)  # canonical batches: edge order
    OC = H * C if concat else C
    bias = torch.randn(OC, device=dev)
    y, ps = ops.gat_attn_fwd(xs, ae, None, bias, None, 1.0, B, n, H, C, concat, 1, 0.2, True)
    dy = torch.randn_like(y)
    tf = bench(lambda: ops.gat_attn_fwd(xs, ae, None, bias, None, 1.0, B, n, H, C, concat, 1, 0.2,
                                        True))
    tb = bench(lambda: ops.gat_attn_bwd(dy, y, xs, ps, None, 1.0, None, True, B, n, H, C, concat,
                                        1, 0.2, True))
    print(f"{name}: target {os.environ.get('SV2N_ATT_TARGET_WG', '1024')}: fwd {tf:.1f} us  "
          f"bwd {tb:.1f} us", flush=True)
