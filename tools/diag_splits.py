"""Per-tensor errors of GATConv (sv2n) vs the fp32 / fp64 oracle for batch
sizes / head counts around the attention split thresholds (diagnostic)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from helpers import block_graphs, float64_twin, max_err, twin_conv  # noqa: E402


def run(B, H, C, concat, dev):
    n = 30
    mine, ref = twin_conv(12, C, H, concat, 3, seed=B + H)
    torch.manual_seed(B)
    x = torch.randn(B * n, 12)
    ei = block_graphs(B, n)
    ea = torch.randn(ei.size(1), 3)
    ref64 = float64_twin(ref)
    mine = mine.to(dev)
    xg = x.clone().to(dev).requires_grad_(True)
    xr = x.clone().requires_grad_(True)
    x64 = x.clone().double().requires_grad_(True)
    out = mine(xg, ei.to(dev), ea.to(dev))
    rout = ref(xr, ei, ea)
    r64 = ref64(x64, ei, ea.double())
    w = torch.randn_like(rout)
    (out * w.to(dev)).sum().backward()
    (rout * w).sum().backward()
    (r64 * w.double()).sum().backward()
    errs = {"fwd": max_err(out, rout), "dx": max_err(xg.grad, xr.grad)}
    for (name, p), (_, q) in zip(mine.named_parameters(), ref.named_parameters()):
        errs[name] = max_err(p.grad, q.grad)
    bad = (xg.grad.cpu() - xr.grad).abs().amax(1)
    rows = torch.nonzero(bad > 1e-4).flatten()
    print(B, H, C, concat, {k: f"{v:.1e}" for k, v in errs.items()},
          "bad rows", rows[:12].tolist(), "graphs", sorted(set((rows // n).tolist()))[:12],
          flush=True)


if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    for cfg in [(1100, 8, 4, True), (1100, 4, 4, True), (1024, 8, 4, True), (1000, 8, 4, True),
                (600, 8, 4, True), (1100, 6, 4, True), (3, 8, 4, True)]:
        run(*cfg, dev)
