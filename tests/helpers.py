"""Shared test helpers: tolerance rule, twin (product, oracle) construction,
random graph batches and keep-mask conversion."""
from __future__ import annotations

import torch

# Tolerance (BASELINE.json north_star: "within 1e-5 fp32"): max |got - ref|
# must be <= TOL * max(1, max |ref|), i.e. absolute 1e-5 for O(1) outputs and
# relative to the largest entry for gradients that sum over many rows.
TOL = 1e-5


def max_err(got: torch.Tensor, ref: torch.Tensor) -> float:
    got = got.detach().double().cpu()
    ref = ref.detach().double().cpu()
    assert got.shape == ref.shape, (got.shape, ref.shape)
    scale = max(1.0, ref.abs().max().item()) if ref.numel() else 1.0
    return (got - ref).abs().max().item() / scale if ref.numel() else 0.0


def assert_parity(got, ref32, ref64, tol=TOL, what=""):
    """Parity with the fp32 reference restatement: |got - ref32| <= tol (scaled),
    OR — where the fp32 reference itself drifts from float64 truth (gradients
    formed by cancellation, e.g. Σ_j of softmax-backward terms that sum to 0
    when negative_slope -> 1) — got is at least as close to the float64
    restatement as the fp32 reference is."""
    if got is None or ref32 is None:
        assert got is None and ref32 is None and ref64 is None, f"{what}: gradient presence"
        return 0.0
    e32 = max_err(got, ref32)
    if e32 <= tol:
        return e32
    e_mine = max_err(got, ref64)
    e_ref = max_err(ref32, ref64)
    assert e_mine <= max(tol, e_ref), (
        f"{what}: |got-ref32| {e32:.3e} > {tol:.1e} and |got-ref64| {e_mine:.3e} > "
        f"|ref32-ref64| {e_ref:.3e}")
    return e32


def float64_twin(ref):
    import copy
    r64 = copy.deepcopy(ref).double()
    return r64


def assert_close(got, ref, tol=TOL, what=""):
    if got is None or ref is None:
        assert got is None and ref is None, f"{what}: one side has no gradient"
        return 0.0
    e = max_err(got, ref)
    assert e <= tol, f"{what}: scaled max error {e:.3e} > {tol:.1e}"
    return e


def twin_conv(in_ch, out_ch, heads, concat, edge_dim, slope=0.2, dropout=0.0, seed=0, bias=True):
    from oracle.pyg_gatconv import OracleGATConv
    from spotv2net_amd import GATConv
    torch.manual_seed(seed)
    mine = GATConv(in_ch, out_ch, heads=heads, concat=concat, edge_dim=edge_dim,
                   negative_slope=slope, dropout=dropout, bias=bias)
    torch.manual_seed(seed)
    ref = OracleGATConv(in_ch, out_ch, heads=heads, concat=concat, edge_dim=edge_dim,
                        negative_slope=slope, dropout=dropout, bias=bias)
    ref.load_state_dict(mine.state_dict())
    # non-zero bias so the bias path is exercised
    with torch.no_grad():
        if mine.bias is not None:
            b = torch.randn_like(mine.bias) * 0.1
            mine.bias.copy_(b)
            ref.bias.copy_(b)
    return mine, ref


def twin_model(seed=0, **kw):
    from oracle.pyg_gatconv import OracleGATModel
    from spotv2net_amd import GATModel
    torch.manual_seed(seed)
    mine = GATModel(**kw)
    torch.manual_seed(seed)
    ref = OracleGATModel(**kw)
    ref.load_state_dict(mine.state_dict())
    return mine, ref


def block_graphs(B, n, keep_frac=1.0, shuffle=False, self_loops=False, seed=0):
    """edge_index of B n-node graphs (canonical order unless shuffled/subset)."""
    from spotv2net_amd.layout import canonical_edge_index
    g = torch.Generator().manual_seed(seed)
    ei = canonical_edge_index(n, B).clone()
    if keep_frac < 1.0:
        m = torch.rand(ei.size(1), generator=g) < keep_frac
        ei = ei[:, m]
    if self_loops:
        loops = torch.arange(0, B * n, 3).repeat(2, 1)
        ei = torch.cat([ei, loops], 1)
    if shuffle:
        ei = ei[:, torch.randperm(ei.size(1), generator=g)]
    return ei.contiguous()


def dense_keep_to_edges(keep, edge_index, n):
    """[B,H,n,n] keep mask -> PyG edge order after remove/add self loops: [E', H]."""
    B, H = keep.shape[:2]
    N = B * n
    ei = edge_index[:, edge_index[0] != edge_index[1]]
    src, dst = ei[0], ei[1]
    g = dst // n
    rows = [keep[g, :, dst - g * n, src - g * n]]
    t = torch.arange(N)
    gl = t // n
    rows.append(keep[gl, :, t - gl * n, t - gl * n])
    return torch.cat(rows, 0).float()
