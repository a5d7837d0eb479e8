"""GPU parity of GATModel (reference utils/models.py surface) against the
oracle GATModel, including the BASELINE configs' full feature widths."""
import pytest
import torch

from helpers import assert_close, assert_parity, float64_twin, twin_model

pytestmark = pytest.mark.gpu


def _check(mine, ref, data, dev):
    from spotv2net_amd import Data
    ref64 = float64_twin(ref)
    mine = mine.to(dev)
    gd = data.to(dev)
    out = mine(gd)
    rout = ref(Data(x=data.x, edge_index=data.edge_index, edge_attr=data.edge_attr))
    r64 = ref64(Data(x=data.x.double(), edge_index=data.edge_index,
                     edge_attr=data.edge_attr.double()))
    assert out.shape == rout.shape
    torch.nn.functional.mse_loss(out, gd.y_x).backward()
    torch.nn.functional.mse_loss(rout, data.y_x).backward()
    torch.nn.functional.mse_loss(r64, data.y_x.double()).backward()
    assert_parity(out, rout, r64, what="forward")
    for (name, p), (_, q), (_, q64) in zip(mine.named_parameters(), ref.named_parameters(),
                                           ref64.named_parameters()):
        assert_parity(p.grad, q.grad, q64.grad, what=f"d{name}")


@pytest.mark.parametrize("act", ["relu", "tanh", "sigmoid"])
def test_c2_shapes_small_batch(dev, act):
    """C2 model (S=42: F=1260, D=126; hidden [100, 50], 4 heads, concat)."""
    from spotv2net_amd import synthetic_batch
    S = 42
    mine, ref = twin_model(seed=5154, num_node_features=30 * S, num_edge_features=3 * S,
                           num_heads=4, output_node_channels=1, dim_hidden_layers=[100, 50],
                           activation=act, concat_heads=True)
    _check(mine, ref, synthetic_batch(6, S, seed=2), dev)


def test_c1_shapes(dev):
    """C1: 1 layer, 1 head, hidden 500 (mean since L == 1)."""
    from spotv2net_amd import synthetic_batch
    S = 42
    mine, ref = twin_model(seed=1, num_node_features=30 * S, num_edge_features=3 * S,
                           num_heads=1, output_node_channels=1, dim_hidden_layers=[500])
    _check(mine, ref, synthetic_batch(4, S, seed=3), dev)


def test_c3_yaml_model(dev):
    """C3: config/GNN_param.yaml model block (hidden [500], 6 heads, concat_heads)."""
    from spotv2net_amd import synthetic_batch
    S = 42
    mine, ref = twin_model(seed=5154, num_node_features=30 * S, num_edge_features=3 * S,
                           num_heads=6, output_node_channels=1, dim_hidden_layers=[500],
                           concat_heads=True)
    _check(mine, ref, synthetic_batch(3, S, seed=4), dev)


@pytest.mark.parametrize("hidden,concat,heads", [([50, 25, 12], True, 3), ([20, 10], False, 4),
                                                 ([16, 16, 16], True, 1)])
def test_deeper_stacks(dev, hidden, concat, heads):
    from spotv2net_amd import synthetic_batch
    S = 3
    mine, ref = twin_model(seed=7, num_node_features=30 * S, num_edge_features=3 * S,
                           num_heads=heads, output_node_channels=2, dim_hidden_layers=hidden,
                           concat_heads=concat, negative_slope=0.1)
    data = synthetic_batch(5, S, seed=5)
    data.y_x = torch.randn(5 * 30 * 2)
    _check(mine, ref, data, dev)


def test_standardize_eval(dev):
    """standardize=True (BatchNorm1d, affine=False) in eval mode."""
    from spotv2net_amd import synthetic_batch
    S = 4
    mine, ref = twin_model(seed=8, num_node_features=30 * S, num_edge_features=3 * S,
                           num_heads=2, output_node_channels=1, dim_hidden_layers=[12, 6],
                           concat_heads=True, standardize=True)
    with torch.no_grad():
        for m in (mine, ref):
            m.bnorm_node.running_mean.fill_(0.1)
            m.bnorm_node.running_var.fill_(2.0)
            m.bnorm_edge.running_mean.fill_(-0.2)
            m.bnorm_edge.running_var.fill_(0.5)
    mine.eval()
    ref.eval()
    _check(mine, ref, synthetic_batch(3, S, seed=6), dev)


def test_c2_full_batch_properties(dev):
    """B=512 (the bench workload): each graph's output equals that graph run
    alone (graphs are independent), and the run is deterministic."""
    from spotv2net_amd import GATModel, synthetic_batch, window_batch
    S = 42
    torch.manual_seed(0)
    model = GATModel(30 * S, 3 * S, 4, 1, [100, 50], concat_heads=True).to(dev)
    data = synthetic_batch(512, S, seed=9, device=dev)
    with torch.no_grad():
        out = model(data)
        out2 = model(data)
        assert torch.equal(out, out2)
        from spotv2net_amd.data import synthetic_series
        V, W = synthetic_series(512 * (S + 1), 30, 9, dev)
        for g in (0, 137, 511):
            one = window_batch(V, W, torch.tensor([g * (S + 1)], device=dev), S)
            o1 = model(one)
            assert_close(o1, out[g * 30:(g + 1) * 30], what=f"graph {g} alone vs batched")


def test_evaluate_matches_notebook_metrics(dev):
    """spotv2net_amd.evaluate reproduces 6_results.ipynb's eval cells (batch-mean
    MSE of de-standardised predictions, elementwise QLIKE) against the oracle
    model evaluated the same way on CPU, and checkpoints round-trip through
    torch.save / load_checkpoint (weights_only)."""
    import os
    import tempfile

    from oracle.pyg_gatconv import OracleGATModel
    from spotv2net_amd import GATModel, WindowDataset, synthetic_series
    from spotv2net_amd.evaluate import evaluate, load_checkpoint, qlike
    S, n = 4, 30
    V, W = synthetic_series(40, n, seed=3)
    ds_cpu = WindowDataset(V, W, S)
    ds_gpu = WindowDataset(V.to(dev), W.to(dev), S)
    torch.manual_seed(2)
    ref = OracleGATModel(n * S, 3 * S, 4, 1, [8, 4], concat_heads=True)
    mine = GATModel(n * S, 3 * S, 4, 1, [8, 4], concat_heads=True)
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "GAT_weights_seed_5154.pth")
        torch.save(ref.state_dict(), path)
        load_checkpoint(mine, path)
    mine = mine.to(dev)
    scaler = (10.0, 2.0)
    got = evaluate(mine, ds_gpu.loader(7, shuffle=False), scaler)
    ref.eval()
    tot, nb, ps, ys = 0.0, 0, [], []
    with torch.no_grad():
        for b in ds_cpu.loader(7, shuffle=False):
            yh = ref(b) * scaler[1] + scaler[0]
            y = b.y_x * scaler[1] + scaler[0]
            tot += torch.nn.functional.mse_loss(yh, y)
            nb += 1
            ps.append(yh)
            ys.append(y)
    assert abs(got.mse - float(tot / nb)) <= 1e-5 * max(1.0, float(tot / nb))
    q = qlike(torch.cat(ys), torch.cat(ps))
    assert_parity(got.qlike, q, q.double(), what="qlike")
    assert abs(got.qlike_mean - float(q.mean())) < 1e-5
