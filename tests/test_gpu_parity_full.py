"""Oracle parity at the sizes the bench runs (BASELINE.json configs C2, C3,
C5), the multi-output head on multi-output windows and the
device-side window builder (§8f-f2).  Tolerance: tests/helpers.py
(1e-5 scaled by max(1, |ref|), or at least as close to the float64
restatement as the fp32 restatement is)."""
import pytest
import torch

from helpers import assert_parity, float64_twin, twin_model

pytestmark = pytest.mark.gpu


def _relu_masks(mine, gd):
    """The active side of every layer's relu in the product's forward (the
    fused stack's saved post-activation outputs, stack.stack_forward)."""
    from spotv2net_amd.model import _layout_of
    from spotv2net_amd.stack import stack_forward
    L = len(mine.gat_layers)
    with torch.no_grad():
        _, saved, _ = stack_forward(gd.x, gd.edge_attr, tuple(mine.gat_layers),
                                    _layout_of(gd, gd.x, gd.edge_index), mine._act_code, 0.0,
                                    False, "f32", True)
    return [(y > 0).cpu() for y in saved[2 + 2 * L:2 + 3 * L]]


def _check_kinks(ref64, masks):
    """The injected relu masks differ from the float64 oracle's own only where
    its pre-activation is within rounding of the kink."""
    for i, (z, m) in enumerate(zip(ref64.act_inputs, masks)):
        diff = (z > 0) != m
        if diff.any():
            worst = z[diff].abs().max().item()
            assert worst <= 1e-5 * max(1.0, z.abs().max().item()), \
                f"layer {i}: relu sides differ at |z| = {worst:.3e}: not a rounding tie"


def _mse_parity(mine, ref, data, dev, post_keep=None, seed=None):
    """Forward + MSE backward on the product (GPU) and the fp32 / fp64 oracle
    (CPU); compare the output and every parameter gradient.  With relu and
    no post-layer dropout the oracle takes the product's relu sides
    (``OracleGATModel.act_masks``): at full batch sizes some pre-activation
    lies within rounding of 0, and the kink's two branches give gradients that
    differ by that node's whole contribution (one such node moves a C2 bias
    gradient by ~1.5e-5); ``_check_kinks`` confirms the sides differ only at
    such ties."""
    from spotv2net_amd import Data
    ref64 = float64_twin(ref)
    if post_keep is not None:
        ref.post_keep = post_keep
        ref64.post_keep = post_keep
    mine = mine.to(dev)
    gd = data.to(dev)
    masks = None
    if ref.activation == "relu" and not ref.dropout:
        masks = _relu_masks(mine, gd)
        ref.act_masks = masks
        ref64.act_masks = masks
    if seed is not None:
        torch.cuda.manual_seed(seed)
    out = mine(gd)
    torch.nn.functional.mse_loss(out, gd.y_x).backward()
    d = Data(x=data.x, edge_index=data.edge_index, edge_attr=data.edge_attr)
    rout = ref(d)
    torch.nn.functional.mse_loss(rout, data.y_x).backward()
    r64 = ref64(Data(x=data.x.double(), edge_index=data.edge_index,
                     edge_attr=data.edge_attr.double()))
    torch.nn.functional.mse_loss(r64, data.y_x.double()).backward()
    if masks is not None:
        _check_kinks(ref64, masks)
    errs = {"forward": assert_parity(out, rout, r64, what="forward")}
    for (name, p), (_, q), (_, q64) in zip(mine.named_parameters(), ref.named_parameters(),
                                           ref64.named_parameters()):
        errs[name] = assert_parity(p.grad, q.grad, q64.grad, what=f"d{name}")
    return errs


def test_c2_full_batch_parity(dev):
    """C2 at the bench's B = 512 (15,360 nodes, 445,440 edges): forward and
    every gradient, including the L0 weight gradient whose split-K GEMM
    reduces K = 15,360 rows."""
    from spotv2net_amd import synthetic_batch
    S = 42
    mine, ref = twin_model(seed=5154, num_node_features=30 * S, num_edge_features=3 * S,
                           num_heads=4, output_node_channels=1, dim_hidden_layers=[100, 50],
                           concat_heads=True)
    _mse_parity(mine, ref, synthetic_batch(512, S, seed=1234), dev)


def test_c5_stress_parity(dev):
    """C5 shapes (256-node dense graphs, S = 4, 3 layers [16,16,16] x 8 heads,
    concat) at B = 4 on the tiled kernels."""
    from spotv2net_amd import synthetic_batch
    S, n = 4, 256
    mine, ref = twin_model(seed=3, num_node_features=n * S, num_edge_features=3 * S,
                           num_heads=8, output_node_channels=1, dim_hidden_layers=[16, 16, 16],
                           concat_heads=True)
    _mse_parity(mine, ref, synthetic_batch(4, S, n=n, seed=77), dev)


def test_c3_yaml_model_with_dropout_parity(dev):
    """config/GNN_param.yaml model as-is (hidden [500], 6 heads, concat_heads,
    dropout 0.1, dropout_att 0.0) in TRAIN mode: the post-layer dropout masks
    the product draws (torch.rand_like(y) >= p, one per layer, on the CUDA
    generator) are regenerated from the same seed and injected into the
    oracle (utils/models.py:148)."""
    from spotv2net_amd import synthetic_batch
    S, B, p = 42, 16, 0.1
    mine, ref = twin_model(seed=5154, num_node_features=30 * S, num_edge_features=3 * S,
                           num_heads=6, output_node_channels=1, dim_hidden_layers=[500],
                           concat_heads=True, dropout=p, dropout_att=0.0)
    mine.train()
    ref.train()
    torch.cuda.manual_seed(321)
    keep = [(torch.rand(B * 30, 500, device=dev) >= p).float().cpu()]
    assert 0.85 < float(keep[0].mean()) < 0.95
    _mse_parity(mine, ref, synthetic_batch(B, S, seed=8), dev, post_keep=keep, seed=321)


def test_multioutput_windows_and_head_parity(dev):
    """CovarianceLaggedMultiOutputDataset windows (F = 14
    future steps) built on the device against the restatement of
    utils/dataset.py:316-411 (bit-exact), then GATModel(output_node_channels=14)
    on those batches against the oracle."""
    from oracle.dataset import lagged_windows_multi
    from spotv2net_amd import Data, WindowDataset, collate
    from spotv2net_amd.data import synthetic_series
    S, Fs, T, cut = 4, 14, 40, 5
    V, W = synthetic_series(T, 30, seed=12)
    ref_w = lagged_windows_multi(list(V.double().numpy()), list(W.double().numpy()), S, Fs, cut)
    ds = WindowDataset(V.to(dev), W.to(dev), S, cut=cut, future_steps=Fs)
    assert len(ds) == len(ref_w) == T - S - Fs + 1 - cut
    idx = torch.tensor([0, 3, len(ds) - 1])
    b = ds.batch(idx)
    want = collate([Data(**{k: v for k, v in ref_w[i].items()}) for i in idx.tolist()])
    for key in ("x", "edge_index", "edge_attr", "y_x"):
        assert torch.equal(getattr(b, key).cpu(), getattr(want, key)), key
    mine, ref = twin_model(seed=4, num_node_features=30 * S, num_edge_features=3 * S,
                           num_heads=4, output_node_channels=Fs, dim_hidden_layers=[16, 8],
                           concat_heads=True)
    cpu_b = collate([Data(**ref_w[i]) for i in range(len(ref_w))])
    _mse_parity(mine, ref, cpu_b, dev)


def test_device_window_dataset_matches_restatement(dev):
    """§8f-f2 on the device: WindowDataset over a device-resident series with
    a leading cut (the reference's data_list[8357:], utils/dataset.py:288)
    yields exactly oracle.dataset.lagged_windows' windows."""
    from oracle.dataset import lagged_windows
    from spotv2net_amd import WindowDataset
    from spotv2net_amd.data import synthetic_series
    S, T, cut = 42, 60, 7
    V, W = synthetic_series(T, 30, seed=13)
    ref_w = lagged_windows(list(V.double().numpy()), list(W.double().numpy()), S, cut)
    ds = WindowDataset(V.to(dev), W.to(dev), S, cut=cut)
    assert len(ds) == len(ref_w) == T - S - cut
    got = ds.batch(torch.arange(len(ds)))
    E0 = 870
    for k, r in enumerate(ref_w):
        assert torch.equal(got.x[k * 30:(k + 1) * 30].cpu(), r["x"])
        assert torch.equal(got.edge_attr[k * E0:(k + 1) * E0].cpu(), r["edge_attr"])
        assert torch.equal(got.y_x[k * 30:(k + 1) * 30].cpu(), r["y_x"])


@pytest.mark.parametrize("n,S,Fs", [(30, 42, 1), (30, 4, 14), (7, 3, 2)])
def test_window_gather_kernel_matches_builder(dev, n, S, Fs):
    """sv2n_window_gather (WindowDataset.fill on the device, one launch) is
    bit-exact with the torch-op builder window_batch (itself checked against
    the restatement of utils/dataset.py), including a ragged index set."""
    from spotv2net_amd import WindowDataset
    from spotv2net_amd.data import synthetic_series
    V, W = synthetic_series(S + Fs + 60, n, seed=n + S)
    ds = WindowDataset(V.to(dev), W.to(dev), S, cut=3, future_steps=Fs)
    idx = torch.randperm(len(ds), generator=torch.Generator().manual_seed(1))[:37].to(dev)
    want = ds.batch(idx)
    got = ds.empty_batch(idx.numel())
    ds.fill(got, idx)
    for key in ("x", "edge_attr", "y_x", "edge_index"):
        assert torch.equal(getattr(got, key), getattr(want, key)), key


@pytest.mark.parametrize("n,S,Fs", [(30, 42, 1), (7, 3, 2), (30, 180, 1)])
def test_window_gather_out_of_range_windows_are_nan(dev, n, S, Fs):
    """torch.ops.sv2n.window_gather with starts outside the series (negative,
    or starts + S + F past the last matrix): those windows come back as NaN,
    nothing is read out of bounds, the in-range windows are unchanged (both
    kernels: the LDS row kernel and, at S = 180, the element-wise gather one)."""
    from spotv2net_amd import WindowDataset
    from spotv2net_amd.data import synthetic_series
    T = S + Fs + 10
    V, W = synthetic_series(T, n, seed=3)
    ds = WindowDataset(V.to(dev), W.to(dev), S, future_steps=Fs)
    good = torch.tensor([0, 3, T - S - Fs], device=dev)
    want = ds.empty_batch(3)
    ds.fill(want, good)  # cut 0: window index == start
    starts = torch.tensor([0, -1, 3, T - S - Fs + 1, T - S - Fs, 10 ** 6], device=dev)
    B = starts.numel()
    E0 = n * (n - 1)
    x = torch.empty(B * n, n * S, device=dev)
    ea = torch.empty(B * E0, 3 * S, device=dev)
    y = torch.empty(B * n * Fs, device=dev)
    from spotv2net_amd.layout import canonical_table
    torch.ops.sv2n.window_gather(ds.vol.contiguous(), ds.volvol.contiguous(), starts, S, Fs,
                                 canonical_table(n, dev), x, ea, y)
    torch.cuda.synchronize()
    bad = [1, 3, 5]
    for b in range(B):
        xs, es, ys = x[b * n:(b + 1) * n], ea[b * E0:(b + 1) * E0], y[b * n * Fs:(b + 1) * n * Fs]
        if b in bad:
            assert torch.isnan(xs).all() and torch.isnan(es).all() and torch.isnan(ys).all(), b
        else:
            assert torch.isfinite(xs).all() and torch.isfinite(es).all(), b
    k = {0: 0, 2: 1, 4: 2}
    for b, j in k.items():
        assert torch.equal(x[b * n:(b + 1) * n], want.x[j * n:(j + 1) * n])
        assert torch.equal(ea[b * E0:(b + 1) * E0], want.edge_attr[j * E0:(j + 1) * E0])


@pytest.mark.parametrize("n,S,Fs", [(30, 42, 1), (30, 180, 1)])
def test_negative_window_index_is_nan_with_cut(dev, n, S, Fs):
    """WindowDataset.fill with a cut: a negative batch index is out of range
    (NaN rows), not a window cut + idx read from before the split (ABI 12),
    on both kernels; the in-range indices of the same launch are unchanged."""
    from spotv2net_amd import WindowDataset
    from spotv2net_amd.data import synthetic_series
    V, W = synthetic_series(S + Fs + 40, n, seed=17)
    ds = WindowDataset(V.to(dev), W.to(dev), S, cut=9, future_steps=Fs)
    idx = torch.tensor([2, -1, 0, -9, len(ds) - 1, len(ds)], device=dev)
    got = ds.empty_batch(idx.numel())
    ds.fill(got, idx)
    want = ds.batch(torch.tensor([2, 0, len(ds) - 1]))
    E0 = n * (n - 1)
    for b, j in {0: 0, 2: 1, 4: 2}.items():
        assert torch.equal(got.x[b * n:(b + 1) * n], want.x[j * n:(j + 1) * n])
        assert torch.equal(got.edge_attr[b * E0:(b + 1) * E0], want.edge_attr[j * E0:(j + 1) * E0])
        assert torch.equal(got.y_x[b * n:(b + 1) * n], want.y_x[j * n:(j + 1) * n])
    for b in (1, 3, 5):
        assert torch.isnan(got.x[b * n:(b + 1) * n]).all(), b
        assert torch.isnan(got.edge_attr[b * E0:(b + 1) * E0]).all(), b
        assert torch.isnan(got.y_x[b * n:(b + 1) * n]).all(), b


@pytest.mark.parametrize("n,S,Fs", [(30, 42, 1), (7, 3, 2)])
def test_window_gather_diag_matches_volvol_path(dev, n, S, Fs):
    """sv2n_window_gather_diag (ABI 11) with the series' diagonal given is bit-exact
    with the kernel reading the diagonal from volvol, in-range and NaN windows alike."""
    from spotv2net_amd import WindowDataset
    from spotv2net_amd.data import synthetic_series
    from spotv2net_amd.layout import canonical_table
    T = S + Fs + 50
    V, W = synthetic_series(T, n, seed=11)
    ds = WindowDataset(V.to(dev), W.to(dev), S, cut=2, future_steps=Fs)
    assert ds.diag is not None and ds.diag.shape == (T, n)
    starts = torch.tensor([0, 5, -4, T, 17, T - S - Fs - 2], device=dev)
    B, E0 = starts.numel(), n * (n - 1)
    outs = []
    for diag in (None, ds.diag):
        x = torch.empty(B * n, n * S, device=dev)
        ea = torch.empty(B * E0, 3 * S, device=dev)
        y = torch.empty(B * n * Fs, device=dev)
        torch.ops.sv2n.window_gather(ds.vol, ds.volvol, starts, S, Fs, canonical_table(n, dev),
                                     x, ea, y, 2, diag)
        outs.append((x, ea, y))
    for a, b in zip(*outs):
        assert torch.equal(a.isnan(), b.isnan())
        assert torch.equal(a.nan_to_num(), b.nan_to_num())
