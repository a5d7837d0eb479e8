import sys, torch
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
from helpers import twin_conv, block_graphs
for heads, C, n, concat in [(1, 49, 48, True), (1, 64, 48, False), (1, 64, 256, True), (1, 33, 48, True), (1, 47, 48, True)]:
    mine, ref = twin_conv(20, C, heads, concat, 3, seed=C)
    ei = block_graphs(2, n)
    x = torch.randn(2 * n, 20); ea = torch.randn(ei.size(1), 3)
    out = mine.cuda()(x.cuda(), ei.cuda(), ea.cuda()).cpu()
    r = ref(x, ei, ea)
    err = (out - r).abs().nan_to_num(1e9)
    print(heads, C, n, concat, "maxerr", float(err.max()), "row0 got", out[0, :4].tolist(), "ref", r[0, :4].tolist(),
          "col err", [round(float(err[:, c].max()), 4) for c in range(0, C, 8)])
