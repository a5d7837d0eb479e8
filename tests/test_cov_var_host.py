"""Host logic of the covariance-layout-only gather (no GPU): when
stack.cov_var_edges_only lets train.Fit gather just the columns the
covariance-layout edge passes read, and the edge-attr marker."""
import torch

from spotv2net_amd import GATModel
from spotv2net_amd.layout import check_full_edge_attr, mark_cov_var_only
from spotv2net_amd.stack import cov_var_edges_only


def test_cov_var_edges_only_conditions():
    c3 = GATModel(30 * 42, 3 * 42, 6, 1, [500], dropout=0.1)
    assert cov_var_edges_only(list(c3.gat_layers), 30, 42)
    assert not cov_var_edges_only(list(c3.gat_layers), 64, 42)     # tiled graphs
    assert not cov_var_edges_only(list(c3.gat_layers), 30, 66)     # window too long
    assert not cov_var_edges_only(list(c3.gat_layers), 30, 41)     # odd S: round-4 passes
    wide = GATModel(120, 12, 8, 1, [8, 8, 8], concat_heads=True)   # L·H = 24 > 16
    assert not cov_var_edges_only(list(wide.gat_layers), 30, 4)


def test_cov_var_only_marker_is_permanent():
    ea = torch.zeros(10, 6)
    check_full_edge_attr(ea, "x")          # unmarked: fine
    mark_cov_var_only(ea)
    ea.add_(1.0)                           # an in-place write keeps the flag
    try:
        check_full_edge_attr(ea, "the test reader")
    except RuntimeError as e:
        assert "the test reader" in str(e)
    else:
        raise AssertionError("a cov-var-only edge_attr was accepted")
