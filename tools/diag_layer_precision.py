"""Diagnostic: gradient accuracy of one GATConv (C2 layer-0-like shapes)
against the PyG-semantics oracle in fp32 and fp64, relative to each
gradient's own magnitude, over a few shape variants — to locate where the
fused path loses precision relative to fp32 PyG."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def run(F, H, C, concat, D, B=32, slope=0.2, seed=0, edge=True):
    from helpers import float64_twin, twin_conv
    from spotv2net_amd.layout import canonical_edge_index
    dev = torch.device("cuda", 0)
    mine, ref = twin_conv(F, C, H, concat, D if edge else None, slope=slope, seed=seed)
    ref64 = float64_twin(ref)
    g = torch.Generator().manual_seed(seed + 1)
    n = 30
    x = torch.randn(B * n, F, generator=g)
    ei = canonical_edge_index(n, B)
    ea = torch.randn(ei.size(1), D, generator=g) if edge else None
    dy = torch.randn(B * n, H * C if concat else C, generator=g)
    mine = mine.to(dev)
    out = mine(x.to(dev), ei.to(dev), ea.to(dev) if edge else None)
    out.backward(dy.to(dev))
    o32 = ref(x, ei, ea)
    o32.backward(dy)
    o64 = ref64(x.double(), ei, ea.double() if edge else None)
    o64.backward(dy.double())
    res = {"out": [(out.detach().double().cpu() - o64.detach()).abs().max().item(),
                   (o32.detach().double() - o64.detach()).abs().max().item(),
                   o64.abs().max().item()]}
    for (name, p), (_, q), (_, r) in zip(mine.named_parameters(), ref.named_parameters(),
                                         ref64.named_parameters()):
        if p.grad is None:
            continue
        gm, g32, g64 = p.grad.double().cpu(), q.grad.double(), r.grad
        res[name] = [(gm - g64).abs().max().item(), (g32 - g64).abs().max().item(),
                     g64.abs().max().item()]
    return res


def main():
    cases = [
        dict(F=1260, H=4, C=100, concat=True, D=126),
        dict(F=1260, H=4, C=100, concat=False, D=126),
        dict(F=400, H=4, C=50, concat=False, D=126),
        dict(F=1260, H=1, C=100, concat=True, D=126),
        dict(F=128, H=4, C=100, concat=True, D=126),
        dict(F=1260, H=4, C=100, concat=True, D=126, edge=False),
        dict(F=1260, H=4, C=100, concat=True, D=126, slope=0.8),
    ]
    for c in cases:
        res = run(**c)
        print(c)
        for k, (em, e32, mag) in res.items():
            print(f"   {k:18s} |ref| {mag:.2e}  mine {em:.2e} ({em / max(mag, 1e-30):.1e} rel)"
                  f"  fp32 PyG {e32:.2e} ({e32 / max(mag, 1e-30):.1e} rel)  ratio {em / max(e32, 1e-30):.0f}")
        sys.stdout.flush()


if __name__ == "__main__":
    main()
