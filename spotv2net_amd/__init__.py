"""spotv2net_amd — MI355X-native SpotV2Net GAT hot path.

Drop-in replacements for the reference's ``GATModel`` (utils/models.py) and the
PyG ``GATConv`` it stacks, running on hand-written gfx950 kernels behind the
C-ABI in ``include/sv2n.h``, plus the PyG-free data containers the reference
training loop needs.
"""
from .conv import GATConv, Linear
from .data import Batch, Data, WindowDataset, collate, shard_indices, synthetic_batch, \
    synthetic_series, window_batch, window_graph
from .layout import GraphLayout, UnsupportedLayout, analyze_edge_index, canonical_edge_index
from .model import GATModel
from . import evaluate, series

__all__ = [
    "GATConv", "GATModel", "Linear", "Data", "Batch", "collate", "window_graph", "window_batch",
    "synthetic_batch", "synthetic_series", "WindowDataset", "GraphLayout", "UnsupportedLayout",
    "analyze_edge_index", "canonical_edge_index", "shard_indices",
]
