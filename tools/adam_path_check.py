"""Which torch.optim.Adam implementation the reference loop gets on this box
(fused / foreach / single-tensor) with GATModel's graph-replayed gradients."""
import os
import sys

import torch
import torch.optim.adam as adam_mod

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from spotv2net_amd import Batch, synthetic_batch  # noqa: E402

calls = []
for fn in ("_single_tensor_adam", "_multi_tensor_adam", "_fused_adam"):
    orig = getattr(adam_mod, fn)

    def w(*a, _o=orig, _n=fn, **k):
        calls.append((_n, k.get("foreach"), len(a[0])))
        return _o(*a, **k)
    setattr(adam_mod, fn, w)
dev = torch.device("cuda", 0)
m = bench.build_model(dev)
opt = torch.optim.Adam(m.parameters(), lr=1e-3)
d = synthetic_batch(64, 42, seed=1, device=dev)
for i in range(4):
    b = Batch(x=d.x, edge_index=d.edge_index.clone(), edge_attr=d.edge_attr, y_x=d.y_x,
              batch=d.batch, ptr=d.ptr, nodes_per_graph=30, canonical_edges=True)
    loss = torch.nn.functional.mse_loss(m(b), b.y_x)
    opt.zero_grad()
    loss.backward()
    opt.step()
    print(i, calls[-1:], opt.param_groups[0].get("foreach"),
          sorted({(tuple(p.grad.stride()) == tuple(p.stride()), p.grad.is_contiguous()) for p in m.parameters()}))
