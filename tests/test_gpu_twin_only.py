"""Twin-only windows (data.WindowDataset.empty_batch(twin_only=True), ABI 21):
the device gather writes bf16(x) alone, x stays NaN, and the bf16 stack's
layer 0 reads x only through the twin.  The training loop on such batches is
bitwise the loop on fully written batches; every path that would read the
fp32 x refuses the batch."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu

S = 42


def _ds(dev, n=30, T=200):
    from spotv2net_amd import WindowDataset
    from spotv2net_amd.data import synthetic_series
    V, W = synthetic_series(T + S, n, seed=99)
    return WindowDataset(V.to(dev), W.to(dev), S)


def test_twin_only_gather_writes_the_same_twin(dev):
    from spotv2net_amd.data import bf16_twin, twin_only_x
    ds = _ds(dev)
    idx = torch.arange(3, 3 + 48, device=dev)
    full = ds.empty_batch(48, bf16_x=True, cov_var_only=True)
    part = ds.empty_batch(48, bf16_x=True, cov_var_only=True, twin_only=True)
    ds.fill(full, idx)
    ds.fill(part, idx)
    torch.cuda.synchronize()
    assert twin_only_x(part) and not twin_only_x(full)
    assert bf16_twin(part) is not None
    assert torch.equal(bf16_twin(part), bf16_twin(full))
    assert torch.isnan(part.x).all()
    assert torch.equal(part.y_x, full.y_x)


def test_twin_only_batch_refused_where_x_is_read(dev):
    from spotv2net_amd import GATModel
    ds = _ds(dev)
    b = ds.empty_batch(48, bf16_x=True, cov_var_only=True, twin_only=True)
    ds.fill(b, torch.arange(48, device=dev))
    torch.manual_seed(1)
    m = GATModel(30 * S, 3 * S, 6, 1, [500], concat_heads=True).to(dev)
    m.graph_replay = False
    with pytest.raises(RuntimeError, match="bf16 twin"):
        m.set_precision("f32")(b)  # fp32 projection of x
    with torch.no_grad():
        out = m.set_precision("bf16")(b)  # the twin GEMM: fine
    assert torch.isfinite(out).all()
    ms = GATModel(30 * S, 3 * S, 6, 1, [500], concat_heads=True, standardize=True).to(dev)
    ms.graph_replay = False
    with pytest.raises(RuntimeError, match="bf16 twin"):
        ms.set_precision("bf16")(b)


def test_fit_twin_only_is_bitwise_full_gather(dev, monkeypatch):
    """Fit on twin-only batches (C3's model, bf16 mode): the loss history and
    the trained parameters are those of the batches with x written."""
    from spotv2net_amd import GATModel, train
    from spotv2net_amd.train import Fit
    ds = _ds(dev)
    torch.manual_seed(11)
    m0 = GATModel(30 * S, 3 * S, 6, 1, [500], concat_heads=True, dropout=0.1).to(dev)
    m0.set_precision("bf16")
    runs = []
    for mode in ("on", "off"):
        monkeypatch.setattr(train, "TWIN_ONLY", mode)
        m = copy.deepcopy(m0)
        torch.manual_seed(5)
        f = Fit(m, ds, 64, generator=torch.Generator().manual_seed(3))
        assert f._cv_only
        assert f._twin_only(64) == (mode == "on")
        assert not f._twin_only(16)  # 480 rows: the rounding GEMM path, x written
        hist = [f.run_epoch() for _ in range(2)]
        runs.append((hist, [p.detach().clone() for p in m.parameters()]))
    (h0, p0), (h1, p1) = runs
    assert h0 == h1
    for a, b in zip(p0, p1):
        assert torch.equal(a, b)
