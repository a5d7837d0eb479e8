"""Times the covariance-layout edge passes against the generic ones on the
C2 batch (HIP events, back to back), for rocprofv3 counter passes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spotv2net_amd  # noqa: E402,F401
from spotv2net_amd import synthetic_batch  # noqa: E402
from spotv2net_amd.layout import canonical_table  # noqa: E402

dev = torch.device("cuda:0")
B, S, n, L, H, hp = 512, 42, 30, 2, 4, 16
b = synthetic_batch(B, S, n=n, seed=1, device=dev)
canon = canonical_table(n, dev)
wf = torch.randn(3 * S, hp, device=dev) * 0.1
ops = torch.ops.sv2n
daes = [torch.randn(B * n * (n - 1), H, device=dev) for _ in range(L)]
runs = {
    "fwd_cv": lambda: ops.edge_logits_cv(b.edge_attr, wf, canon, L, H, B, n),
    "fwd_mx": lambda: ops.edge_logits(b.edge_attr, wf, None, canon, L, H, B, n, False),
    "bwd_cv": lambda: ops.edge_logits_bwd_cv(b.edge_attr, canon, daes, H, B, n, hp),
    "bwd_mx": lambda: ops.edge_logits_bwd(b.edge_attr, None, canon, daes, H, B, n, hp, False),
}
for name, fn in runs.items():
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"{name}: {e0.elapsed_time(e1) * 1e3 / 20:.1f} us")
