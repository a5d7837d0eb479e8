import sys, torch
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
from helpers import twin_conv, block_graphs, max_err
from oracle.pyg_gatconv import OracleGATConv
dev = torch.device('cuda:0')
for slope, scale in [(0.2, 1), (0.8, 3), (0.8, 1), (0.05, 3)]:
    mine, ref = twin_conv(12, 6, 3, False, 4, slope=slope, seed=8)
    ref64 = OracleGATConv(12, 6, heads=3, concat=False, edge_dim=4, negative_slope=slope).double()
    ref64.load_state_dict({k: v.double() for k, v in ref.state_dict().items()})
    torch.manual_seed(0)
    x = torch.randn(60, 12) * scale
    ei = block_graphs(2, 30); ea = torch.randn(ei.size(1), 4)
    mine = mine.to(dev)
    out = mine(x.to(dev), ei.to(dev), ea.to(dev)); r = ref(x, ei, ea); r64 = ref64(x.double(), ei, ea.double())
    w = torch.randn_like(r)
    (out * w.to(dev)).sum().backward(); (r*w).sum().backward(); (r64*w.double()).sum().backward()
    print(f"slope {slope} scale {scale}: fwd mine-64 {max_err(out, r64):.2e} ref32-64 {max_err(r, r64):.2e}")
    for (nm, p), (_, q), (_, q64) in zip(mine.named_parameters(), ref.named_parameters(), ref64.named_parameters()):
        print(f"   {nm:18s} mine-64 {max_err(p.grad, q64.grad):.2e}  ref32-64 {max_err(q.grad, q64.grad):.2e}  mine-ref32 {max_err(p.grad, q.grad):.2e}")
