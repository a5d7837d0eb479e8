"""Diagnostic: where a library build's fused-attention backward goes non-finite.
python tools/diag_fused_nan.py OUT.pt n H C D concat (SV2N_LIB selects the build)."""
import sys
import torch
sys.path[:0] = [".", "tests"]
from helpers import block_graphs, twin_conv  # noqa: E402

out, n, H, C, D, concat = sys.argv[1], *map(int, sys.argv[2:6]), sys.argv[6] == "1"
dev = "cuda"
B = 2
mine, ref = twin_conv(20, C, H, concat, D, seed=n + H)
torch.manual_seed(n)
ei = block_graphs(B, n)
x = torch.randn(B * n, 20)
ea = torch.randn(ei.size(1), D)
mine = mine.to(dev)
xg = x.clone().to(dev).requires_grad_(True)
y = mine(xg, ei.to(dev), ea.to(dev))
w = torch.randn(y.shape)
(y * w.to(dev)).sum().backward()
res = {"y": y.detach().cpu(), "dx": xg.grad.cpu()}
for k, p in mine.named_parameters():
    res["d" + k] = p.grad.cpu()
torch.save(res, out)
for k, v in res.items():
    bad = ~torch.isfinite(v)
    print(k, tuple(v.shape), "nonfinite", int(bad.sum()),
          "rows" if v.dim() > 1 else "", bad.any(dim=-1).nonzero().flatten()[:20].tolist() if v.dim() > 1 else "")
