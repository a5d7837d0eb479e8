"""CPU checks of the window builders (reference utils/dataset.py) and of the
host-side argument validation; no GPU work."""
import pytest
import torch


def test_multioutput_windows_match_restatement():
    """window_batch(future_steps=F) vs the restatement of
    CovarianceLaggedMultiOutputDataset.process (utils/dataset.py:316-411),
    including the leading cut (:411)."""
    from oracle.dataset import lagged_windows_multi
    from spotv2net_amd import WindowDataset
    from spotv2net_amd.data import synthetic_series
    n, S, T, Fs, cut = 5, 3, 14, 4, 2
    V, W = synthetic_series(T, n, seed=3, dtype=torch.float64)
    ref = lagged_windows_multi(list(V.numpy()), list(W.numpy()), S, Fs, cut)
    ds = WindowDataset(V, W, S, cut=cut, future_steps=Fs)
    assert len(ds) == len(ref) == T - S - Fs + 1 - cut
    b = ds.batch(torch.arange(len(ds)))
    E0 = n * (n - 1)
    for k, r in enumerate(ref):
        assert torch.equal(b.x[k * n:(k + 1) * n], r["x"])
        assert torch.equal(b.edge_attr[k * E0:(k + 1) * E0], r["edge_attr"])
        assert torch.equal(b.edge_index[:, k * E0:(k + 1) * E0] - k * n, r["edge_index"])
        assert torch.equal(b.y_x[k * n * Fs:(k + 1) * n * Fs], r["y_x"])


def test_single_output_is_future_steps_one():
    """future_steps=1 of the multi-output builder == the single-output
    CovarianceLaggedDataset target (same windows, same y_x)."""
    from oracle.dataset import lagged_windows, lagged_windows_multi
    from spotv2net_amd.data import synthetic_series
    V, W = synthetic_series(9, 4, seed=4, dtype=torch.float64)
    a = lagged_windows(list(V.numpy()), list(W.numpy()), 3)
    b = lagged_windows_multi(list(V.numpy()), list(W.numpy()), 3, 1)
    assert len(a) == len(b)
    for u, v in zip(a, b):
        for key in ("x", "edge_attr", "y_x"):
            assert torch.equal(u[key], v[key])


def test_window_dataset_with_cut_matches_restatement():
    """WindowDataset(cut=c) keeps the reference's data_list[c:] (utils/dataset.py:288)."""
    from oracle.dataset import lagged_windows
    from spotv2net_amd import WindowDataset
    from spotv2net_amd.data import synthetic_series
    n, S, T, cut = 4, 2, 11, 3
    V, W = synthetic_series(T, n, seed=5, dtype=torch.float64)
    ref = lagged_windows(list(V.numpy()), list(W.numpy()), S, cut)
    ds = WindowDataset(V, W, S, cut=cut)
    b = ds.batch(torch.arange(len(ds)))
    assert len(ds) == len(ref)
    for k, r in enumerate(ref):
        assert torch.equal(b.x[k * n:(k + 1) * n], r["x"])
        assert torch.equal(b.y_x[k * n:(k + 1) * n], r["y_x"])


def test_c3_window_count():
    """BASELINE C3: 10,556 matrices, S = 42, cut 8357 -> 2,157 windows
    (utils/dataset.py:200, :288); split 0.8 (yaml:6) -> 1,725 / 432."""
    from spotv2net_amd import WindowDataset
    V = torch.zeros(10556, 1, 1)
    ds = WindowDataset(V, V, 42, cut=8357)
    assert len(ds) == 2157
    assert int(0.8 * len(ds)) == 1725


def test_model_double_with_fp32_data_raises():
    """The kernels read parameters as fp32 through raw pointers: a float64
    model must be refused before any kernel (stock PyTorch also raises)."""
    from spotv2net_amd import GATModel, synthetic_batch
    m = GATModel(30 * 2, 3 * 2, 2, 1, [4]).double()
    data = synthetic_batch(1, 2)
    with pytest.raises(TypeError):
        m(data)
    m2 = GATModel(30 * 2, 3 * 2, 2, 1, [4])
    m2.linear.double()
    from spotv2net_amd.stack import linear_head
    with pytest.raises(TypeError):
        linear_head(torch.randn(30, 4), m2.linear)


def test_collate_marks_canonical_batches():
    """collate checks every graph's edge_index on the host: canonical order
    -> ``canonical_edges`` (no device analysis of the batch); a shuffled graph
    or ragged sizes -> no mark."""
    from spotv2net_amd import Data, collate
    from spotv2net_amd.data import synthetic_series, window_graph
    V, W = synthetic_series(8, 30, seed=1)
    gs = [window_graph(V[k:k + 3], W[k:k + 3]) for k in range(3)]
    assert getattr(collate(gs), "canonical_edges", False)
    ei = gs[1].edge_index[:, torch.randperm(870, generator=torch.Generator().manual_seed(0))]
    bad = [gs[0], Data(x=gs[1].x, edge_index=ei, edge_attr=gs[1].edge_attr, y_x=gs[1].y_x)]
    assert not getattr(collate(bad), "canonical_edges", False)
    small = Data(x=torch.zeros(5, 60), edge_index=torch.zeros(2, 0, dtype=torch.long),
                 edge_attr=torch.zeros(0, 6), y_x=torch.zeros(5))
    assert not getattr(collate([gs[0], small]), "canonical_edges", False)


def test_cov_var_mark_follows_the_tensor_version():
    """layout.mark_cov_var holds for the tensor's current contents only."""
    import torch
    from spotv2net_amd.layout import cov_var_seq_length, mark_cov_var
    ea = torch.zeros(6, 9)
    assert cov_var_seq_length(ea) is None
    mark_cov_var(ea, 3)
    assert cov_var_seq_length(ea) == 3
    ea[0, 0] = 1.0
    assert cov_var_seq_length(ea) is None
    assert cov_var_seq_length(mark_cov_var(torch.zeros(6, 8), 3)) is None  # not 3 x S columns
