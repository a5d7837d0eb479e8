"""PyG-compatible ``GATConv`` running on the sv2n MI355X kernels.

Surface, parameter names and initialisation restate PyG 2.3.0
``torch_geometric.nn.GATConv`` as the reference constructs it
(reference utils/models.py:87-113: ``GATConv(in_channels, out_channels,
heads, concat, dropout, edge_dim, negative_slope)``) and calls it
(utils/models.py:146: ``l(x, edge_index, edge_attr)``).  PyG itself is not part
of the reference tree (imported at utils/models.py:11, pinned to 2.3.0 at
README.md:88) and not installed here, so its semantics are restated from its
published source:

* ``lin_src`` = ``lin_dst``: one bias-free glorot ``Linear(in, H*C)`` (the
  ``lin_dst`` attribute aliases the same module, so state_dict carries both
  ``lin_src.weight`` and ``lin_dst.weight``).
* ``att_src``, ``att_dst``, ``att_edge``: [1, H, C] glorot; ``lin_edge``:
  bias-free glorot ``Linear(edge_dim, H*C)``; ``bias``: [H*C] (concat) or [C],
  zeros.
* forward: self loops removed then re-added with ``fill_value='mean'``
  (grouped by target), logits a_src[j] + a_dst[i] + a_edge[e], leaky_relu,
  softmax per target, attention dropout, scatter-add of p·xs[j], concat or head
  mean, + bias.

Execution differs from PyG, not the math: the node projection carries two extra
GEMM columns per head (W_srcᵀatt_src and W_srcᵀatt_dst, so a_src/a_dst come out
of the projection), and the edge projection is folded to W̃ = W_edgeᵀatt_edge
(one D x H matrix), so ``lin_edge(edge_attr)`` is never materialised.  The
forward and backward run as one fused node (``stack.gat_stack``) whose
backward undoes the folds in-kernel and accumulates into each parameter's
``.grad``.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
from torch import Tensor, nn

from . import ops
from .layout import GraphLayout, analyze_edge_index
from .stack import gat_stack


def glorot_(t: Tensor) -> None:
    """PyG ``inits.glorot``: U(-a, a), a = sqrt(6 / (size(-2) + size(-1)))."""
    a = math.sqrt(6.0 / (t.size(-2) + t.size(-1)))
    with torch.no_grad():
        t.uniform_(-a, a)


class Linear(nn.Module):
    """PyG ``torch_geometric.nn.dense.linear.Linear`` as GATConv uses it:
    ``weight`` [out, in], glorot init, no bias."""

    def __init__(self, in_channels: int, out_channels: int, bias: bool = False):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.weight = nn.Parameter(torch.empty(out_channels, in_channels))
        if bias:
            self.bias = nn.Parameter(torch.empty(out_channels))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self) -> None:
        glorot_(self.weight)
        if self.bias is not None:
            with torch.no_grad():
                self.bias.zero_()

    def forward(self, x: Tensor) -> Tensor:
        y = ops.linear(x, self.weight)
        return y + self.bias if self.bias is not None else y


def fold_edge_weight(lin_edge_weight: Tensor, att_edge: Tensor) -> Tensor:
    """W̃[d, h] = Σ_c W_edge[h*C+c, d] · att_edge[0, h, c]  ->  [D, H]."""
    _, H, C = att_edge.shape
    D = lin_edge_weight.shape[1]
    return torch.einsum("hcd,hc->dh", lin_edge_weight.view(H, C, D), att_edge.view(H, C))


class GATConv(nn.Module):
    def __init__(self, in_channels: int, out_channels: int, heads: int = 1, concat: bool = True,
                 negative_slope: float = 0.2, dropout: float = 0.0, add_self_loops: bool = True,
                 edge_dim: Optional[int] = None, fill_value="mean", bias: bool = True, **kwargs):
        super().__init__()
        if not isinstance(in_channels, int):
            raise NotImplementedError("bipartite (tuple) in_channels are not used by the "
                                      "reference and not supported")
        if not add_self_loops or fill_value != "mean":
            raise NotImplementedError("the reference uses add_self_loops=True, fill_value='mean'")
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.heads = heads
        self.concat = concat
        self.negative_slope = negative_slope
        self.dropout = dropout
        self.add_self_loops = add_self_loops
        self.edge_dim = edge_dim
        self.fill_value = fill_value
        self.precision: Optional[str] = None  # see GATModel.set_precision

        # registration order follows PyG 2.3.0 (state_dict key order)
        self.lin_src = Linear(in_channels, heads * out_channels)
        self.lin_dst = self.lin_src
        self.att_src = nn.Parameter(torch.empty(1, heads, out_channels))
        self.att_dst = nn.Parameter(torch.empty(1, heads, out_channels))
        if edge_dim is not None:
            self.lin_edge = Linear(edge_dim, heads * out_channels)
            self.att_edge = nn.Parameter(torch.empty(1, heads, out_channels))
        else:
            self.lin_edge = None
            self.register_parameter("att_edge", None)
        if bias and concat:
            self.bias = nn.Parameter(torch.empty(heads * out_channels))
        elif bias:
            self.bias = nn.Parameter(torch.empty(out_channels))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self) -> None:
        # PyG 2.3.0 GATConv.reset_parameters (lin_dst is lin_src: re-drawn twice)
        self.lin_src.reset_parameters()
        self.lin_dst.reset_parameters()
        if self.lin_edge is not None:
            self.lin_edge.reset_parameters()
        glorot_(self.att_src)
        glorot_(self.att_dst)
        if self.att_edge is not None:
            glorot_(self.att_edge)
        if self.bias is not None:
            with torch.no_grad():
                self.bias.zero_()

    # ---- building blocks shared with GATModel's fused path ----
    @property
    def out_dim(self) -> int:
        return self.heads * self.out_channels if self.concat else self.out_channels

    def projection_weight(self) -> Tensor:
        """[ldx, in]: rows = lin_src.weight | W_srcᵀatt_src | W_srcᵀatt_dst | 0-pad,
        ldx rounded up to a multiple of 4 (16-B rows)."""
        H, C = self.heads, self.out_channels
        W = self.lin_src.weight
        Wv = W.view(H, C, self.in_channels)
        fs = torch.einsum("hcf,hc->hf", Wv, self.att_src.view(H, C))
        fd = torch.einsum("hcf,hc->hf", Wv, self.att_dst.view(H, C))
        rows = H * C + 2 * H
        ldx = (rows + 3) // 4 * 4
        parts = [W, fs, fd]
        if ldx != rows:
            parts.append(W.new_zeros(ldx - rows, self.in_channels))
        return torch.cat(parts, 0)

    def edge_fold(self) -> Optional[Tensor]:
        if self.lin_edge is None:
            return None
        return fold_edge_weight(self.lin_edge.weight, self.att_edge)

    def forward(self, x: Tensor, edge_index: Tensor, edge_attr: Optional[Tensor] = None,
                size=None, return_attention_weights=None, *,
                layout: Optional[GraphLayout] = None) -> Tensor:
        if return_attention_weights:
            raise NotImplementedError("return_attention_weights is not used by the reference")
        if size is not None:
            raise NotImplementedError("bipartite `size` is not used by the reference")
        if x.dim() != 2:
            raise ValueError("x must be [N, in_channels]")
        if layout is None:
            layout = analyze_edge_index(edge_index, x.size(0))
        return gat_stack(x, edge_attr, (self,), layout, ops.ACT_CODES[None], 0.0, self.training,
                         self.precision)

    def __repr__(self) -> str:
        return (f"{self.__class__.__name__}({self.in_channels}, {self.out_channels}, "
                f"heads={self.heads})")
