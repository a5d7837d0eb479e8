"""Oracle parity at the edges of the reference's HPO grid
(config/GNN_param.yaml:45-64): seq_length up to 120 (F = 3600 node / D = 360
edge features), hidden layers up to [600, 600, 600], up to 7 heads
concatenated (4,200-wide layers), i.e. L·H = 21 edge-logit columns — past the
16 the MFMA and covariance-layout edge passes take, so these shapes run the
generic edge passes (k_edge_fwd / k_edge_bwd with several 4x4 gradient tiles
per thread) and the split n <= 32 attention.  Tolerance: tests/helpers.py.
The supported envelope per kernel path is DESIGN.md §4 "Supported shapes"."""
import pytest
import torch

from helpers import twin_model
from test_gpu_parity_full import _mse_parity

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("S,hidden,heads,concat,act", [
    (120, [600, 600, 600], 7, True, "relu"),     # the grid's widest model, longest window
    (84, [500, 250, 125], 7, True, "relu"),      # L·H = 21, D = 252
    (108, [200, 50], 3, False, "tanh"),          # mean heads, L·H = 6 at D = 324
])
def test_hpo_grid_shapes_match_oracle(dev, S, hidden, heads, concat, act):
    from spotv2net_amd import stack, synthetic_batch
    mine, ref = twin_model(seed=5154, num_node_features=30 * S, num_edge_features=3 * S,
                           num_heads=heads, output_node_channels=1, dim_hidden_layers=hidden,
                           concat_heads=concat, activation=act)
    _mse_parity(mine, ref, synthetic_batch(2, S, seed=17), dev)
    # the batch carries the covariance-layout mark: it takes the covariance
    # passes only where they fit (L·H <= 16, S <= 64)
    assert stack.LAST_PATH["cov_var"] is (len(hidden) * heads <= 16 and S <= 64)
    assert stack.LAST_PATH["attention"] == "small"


def test_hpo_grid_trainstep_batch_512(dev):
    """The grid's largest batch (512) at S = 84 with [500, 250, 125] x 7 heads
    concat: the captured training step runs and equals the eager step bit for
    bit over two Adam steps."""
    import copy

    from spotv2net_amd import GATModel, synthetic_batch
    from spotv2net_amd.train import TrainStep
    S = 84
    torch.manual_seed(5154)
    m1 = GATModel(30 * S, 3 * S, 7, 1, [500, 250, 125], concat_heads=True).to(dev)
    m2 = copy.deepcopy(m1)
    data = synthetic_batch(512, S, seed=3, device=dev)
    s1 = TrainStep(m1, data, lr=1e-3, use_graph=True)
    s2 = TrainStep(m2, data, lr=1e-3, use_graph=False)
    for _ in range(2):
        a, b = float(s1()), float(s2())
        assert a == b and a == a, (a, b)
    for (n, p), (_, q) in zip(m1.named_parameters(), m2.named_parameters()):
        assert torch.equal(p, q), n


def test_edge_columns_past_32_raise(dev):
    """More than 32 edge-logit columns (layers x heads) is outside every edge
    pass: a documented ValueError, not a kernel launch."""
    from spotv2net_amd import GATModel, synthetic_batch
    torch.manual_seed(0)
    m = GATModel(30 * 2, 6, 8, 1, [4, 4, 4, 4, 4], concat_heads=True).to(dev)
    with pytest.raises(ValueError, match="edge-logit columns"):
        m(synthetic_batch(2, 2, seed=1, device=dev))
