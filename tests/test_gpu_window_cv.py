"""The covariance-layout-only window gather (sv2n_window_gather_cv, ABI 19):
``WindowDataset.empty_batch(cov_var_only=True)`` batches carry x, y (and the
bf16 twin) in full but of edge_attr only the columns the covariance-layout
edge passes read; a model reading them through those passes computes the
same bits as on the full gather, and every other edge reader refuses them."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

S = 42


def _ds(dev, T=160):
    from spotv2net_amd import WindowDataset
    from spotv2net_amd.data import synthetic_series
    V, W = synthetic_series(T + S, 30, seed=5)
    return WindowDataset(V.to(dev), W.to(dev), S)


def _cv_columns(n, B):
    """Mask [B*E0][3S] of what sv2n_edge.hip's cv passes read."""
    E0, P = n * (n - 1), n * (n - 1) // 2
    m = torch.zeros(B, E0, 3 * S, dtype=torch.bool)
    m[:, :P, :S] = True                 # covariance columns of the upper rows
    m[:, 0, S:2 * S] = True             # source variance of pair (0, 1)
    m[:, :n - 1, 2 * S:] = True         # target variance of pairs (0, w)
    pad = (16 - P % 16) % 16
    m[:, P:P + pad, :S] = True          # lower rows the passes' last 16-row tile reaches
    return m.view(B * E0, 3 * S)


@pytest.mark.parametrize("bf16_x", [False, True])
def test_cv_gather_writes_what_the_cv_passes_read(dev, bf16_x):
    from spotv2net_amd.data import bf16_twin
    ds = _ds(dev)
    B = 24
    idx = torch.randperm(len(ds), generator=torch.Generator().manual_seed(1))[:B].to(dev)
    full = ds.empty_batch(B, bf16_x=bf16_x)
    ds.fill(full, idx)
    part = ds.empty_batch(B, bf16_x=bf16_x, cov_var_only=True)
    assert getattr(part, "_cov_var_only", False)
    part.edge_attr.fill_(math.nan)
    ds.fill(part, idx)
    torch.cuda.synchronize()
    assert torch.equal(part.x, full.x) and torch.equal(part.y_x, full.y_x)
    if bf16_x:
        assert torch.equal(bf16_twin(part), bf16_twin(full))
    m = _cv_columns(30, B).to(dev)
    assert torch.equal(part.edge_attr[m], full.edge_attr[m])
    assert bool(torch.isnan(part.edge_attr[~m]).all())
    assert m.float().mean().item() < 0.2   # ≈ 1/6 of the edge bytes


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_model_on_cv_batch_is_bitwise_full_batch(dev, precision):
    """forward + backward of a model whose edge path is the covariance-layout
    passes: the same output and gradients on both gathers."""
    from spotv2net_amd import GATModel
    from spotv2net_amd.stack import cov_var_edges_only
    ds = _ds(dev)
    B = 16
    idx = torch.arange(B, device=dev) * 3
    full = ds.empty_batch(B, bf16_x=precision == "bf16")
    ds.fill(full, idx)
    part = ds.empty_batch(B, bf16_x=precision == "bf16", cov_var_only=True)
    part.edge_attr.fill_(math.nan)
    ds.fill(part, idx)
    torch.manual_seed(3)
    m = GATModel(30 * S, 3 * S, 4, 1, [32, 16], concat_heads=True).to(dev)
    if precision == "bf16":
        m.precision = "bf16"
    assert cov_var_edges_only(list(m.gat_layers), 30, S)
    outs, grads = [], []
    for b in (full, part):
        m.zero_grad(set_to_none=True)
        out = m(b)
        (out ** 2).mean().backward()
        outs.append(out.detach())
        grads.append([p.grad.clone() for p in m.parameters()])
    assert torch.equal(outs[0], outs[1])
    for g0, g1 in zip(*grads):
        assert torch.equal(g0, g1)


def test_other_edge_paths_refuse_a_cv_batch(dev, monkeypatch):
    from spotv2net_amd import GATModel, stack
    ds = _ds(dev)
    part = ds.empty_batch(8, cov_var_only=True)
    ds.fill(part, torch.arange(8, device=dev))
    torch.manual_seed(4)
    m = GATModel(30 * S, 3 * S, 4, 1, [16], concat_heads=True).to(dev)
    monkeypatch.setattr(stack, "COV_VAR_EDGES", "off")
    with pytest.raises(RuntimeError, match="covariance-layout"):
        m(part)
    monkeypatch.setattr(stack, "COV_VAR_EDGES", "on")
    ms = GATModel(30 * S, 3 * S, 4, 1, [16], concat_heads=True, standardize=True).to(dev)
    with pytest.raises(RuntimeError, match="BatchNorm"):
        ms(part)
    m(part)  # the covariance-layout path takes it


@pytest.mark.parametrize("n", [2, 3, 5, 17])
def test_cv_batch_small_graphs_bitwise_full_batch(dev, n):
    """Graph sizes whose last 16-pair tile reaches past the upper rows by
    more than the lower rows (n = 2, 3, 5: pad > P) or by a partial tile
    (n = 17): the columns the cv-only gather leaves NaN are never read —
    forward and every gradient equal the full gather's bit for bit."""
    from spotv2net_amd import GATModel, WindowDataset
    from spotv2net_amd.data import synthetic_series
    from spotv2net_amd.stack import cov_var_edges_only
    V, W = synthetic_series(60 + S, n, seed=7)
    ds = WindowDataset(V.to(dev), W.to(dev), S)
    B = 12
    idx = torch.arange(B, device=dev) * 4
    full = ds.empty_batch(B)
    ds.fill(full, idx)
    part = ds.empty_batch(B, cov_var_only=True)
    part.edge_attr.fill_(math.nan)
    ds.fill(part, idx)
    torch.manual_seed(11)
    m = GATModel(n * S, 3 * S, 4, 1, [16, 8], concat_heads=True).to(dev)
    assert cov_var_edges_only(list(m.gat_layers), n, S)
    outs, grads = [], []
    for b in (full, part):
        m.zero_grad(set_to_none=True)
        out = m(b)
        (out ** 2).mean().backward()
        outs.append(out.detach())
        grads.append([p.grad.clone() for p in m.parameters()])
    assert torch.isfinite(outs[0]).all()
    assert torch.equal(outs[0], outs[1])
    for (name, _), g0, g1 in zip(m.named_parameters(), *grads):
        assert torch.equal(g0, g1), name
