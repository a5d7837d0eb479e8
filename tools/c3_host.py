"""Is the C3 loop host-bound?  Times, per epoch of the bench's C3 bf16 Fit:
the wall time (synchronised), the host time spent enqueueing it (up to the
epoch's one loss sync), and the host time of the pieces of one step
(index copy, graph replay) with the GPU kept busy."""
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from spotv2net_amd import WindowDataset  # noqa: E402
from spotv2net_amd.data import synthetic_series  # noqa: E402
from spotv2net_amd.train import Fit  # noqa: E402

dev = torch.device("cuda:0")
cfg = bench.CONFIGS["c3"]
V, W = synthetic_series(10556, cfg["n"], seed=1234, device=dev)
ds = WindowDataset(V, W, cfg["S"], cut=8357)
model = bench.build_model(dev, cfg).set_precision("bf16")
f = Fit(model, ds, cfg["batch"], lr=1e-3, split=0.8, generator=torch.Generator().manual_seed(5))
for _ in range(2):
    f.run_epoch()
torch.cuda.synchronize()
for _ in range(3):
    t0 = time.perf_counter()
    f.run_epoch()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"epoch wall {1e3 * (t1 - t0):.3f} ms (includes the loss sync)")
b = cfg["batch"]
idx = f._idx[b]
perm = torch.arange(b, device=dev)
sh = f._train_shape[b]
# host cost of the pieces, GPU saturated by a long queue first
for name, fn in (("idx copy", lambda: idx.copy_(perm)), ("replay", lambda: f.step(sh)),
                 ("copy+replay", lambda: (idx.copy_(perm), f.step(sh)))):
    torch.cuda.synchronize()
    n = 50
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{name}: host {1e6 * (t1 - t0) / n:.1f} us/call, wall {1e6 * (t2 - t0) / n:.1f} us/call")
