"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py; parity unpinned).

Op-for-op CPU restatement of PyG 2.3.0 ``GATConv`` (third-party; the reference
constructs it at utils/models.py:87-113 and calls it at utils/models.py:146)
and of the reference's ``GATModel`` (utils/models.py:61-152).

PyG 2.3.0 pieces restated (from the published source of that release):
* ``torch_geometric.nn.inits.glorot``: U(-a, a), a = sqrt(6/(size(-2)+size(-1)))
* ``torch_geometric.nn.dense.linear.Linear(weight_initializer='glorot')``:
  weight [out, in], reset in __init__
* ``torch_geometric.utils.remove_self_loops`` / ``add_self_loops`` with
  ``fill_value='mean'`` (scatter-mean of edge_attr grouped by edge_index[1],
  loops appended after the kept edges)
* ``torch_geometric.utils.softmax(src, index, num_nodes)``:
  src_max = scatter(src.detach(), index, reduce='max');
  out = (src - src_max[index]).exp();
  out / (scatter(out, index, reduce='sum')[index] + 1e-16)
* ``GATConv.forward`` / ``edge_update`` / ``message`` with aggr='add'.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn.functional as F
from torch import Tensor, nn


def glorot_(t: Tensor) -> None:
    a = math.sqrt(6.0 / (t.size(-2) + t.size(-1)))
    with torch.no_grad():
        t.uniform_(-a, a)


class PygLinear(nn.Module):
    def __init__(self, in_channels: int, out_channels: int):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(out_channels, in_channels))
        self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        glorot_(self.weight)

    def forward(self, x: Tensor) -> Tensor:
        return F.linear(x, self.weight)


def scatter_sum(src: Tensor, index: Tensor, dim_size: int) -> Tensor:
    out = src.new_zeros((dim_size,) + tuple(src.shape[1:]))
    return out.index_add_(0, index, src)


def scatter_max(src: Tensor, index: Tensor, dim_size: int) -> Tensor:
    out = src.new_zeros((dim_size,) + tuple(src.shape[1:]))
    idx = index.view(-1, *([1] * (src.dim() - 1))).expand_as(src)
    return out.scatter_reduce(0, idx, src, reduce="amax", include_self=False)


def scatter_mean(src: Tensor, index: Tensor, dim_size: int) -> Tensor:
    s = scatter_sum(src, index, dim_size)
    cnt = scatter_sum(torch.ones_like(index, dtype=src.dtype), index, dim_size).clamp(min=1)
    return s / cnt.view(-1, *([1] * (src.dim() - 1)))


def remove_self_loops(edge_index: Tensor, edge_attr: Optional[Tensor]):
    mask = edge_index[0] != edge_index[1]
    return edge_index[:, mask], (edge_attr[mask] if edge_attr is not None else None)


def add_self_loops(edge_index: Tensor, edge_attr: Optional[Tensor], fill_value: str,
                   num_nodes: int):
    loop_index = torch.arange(num_nodes, dtype=torch.long,
                              device=edge_index.device).unsqueeze(0).repeat(2, 1)
    if edge_attr is not None:
        assert fill_value == "mean"
        loop_attr = scatter_mean(edge_attr, edge_index[1], num_nodes)
        edge_attr = torch.cat([edge_attr, loop_attr], dim=0)
    return torch.cat([edge_index, loop_index], dim=1), edge_attr


def pyg_softmax(src: Tensor, index: Tensor, num_nodes: int) -> Tensor:
    src_max = scatter_max(src.detach(), index, num_nodes)
    out = (src - src_max.index_select(0, index)).exp()
    out_sum = scatter_sum(out, index, num_nodes) + 1e-16
    return out / out_sum.index_select(0, index)


class OracleGATConv(nn.Module):
    def __init__(self, in_channels: int, out_channels: int, heads: int = 1, concat: bool = True,
                 negative_slope: float = 0.2, dropout: float = 0.0, add_self_loops: bool = True,
                 edge_dim: Optional[int] = None, fill_value="mean", bias: bool = True):
        super().__init__()
        self.in_channels, self.out_channels, self.heads = in_channels, out_channels, heads
        self.concat, self.negative_slope, self.dropout = concat, negative_slope, dropout
        self.add_self_loops, self.edge_dim, self.fill_value = add_self_loops, edge_dim, fill_value
        self.lin_src = PygLinear(in_channels, heads * out_channels)
        self.lin_dst = self.lin_src
        self.att_src = nn.Parameter(torch.empty(1, heads, out_channels))
        self.att_dst = nn.Parameter(torch.empty(1, heads, out_channels))
        if edge_dim is not None:
            self.lin_edge = PygLinear(edge_dim, heads * out_channels)
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
        # test hook: an explicit attention-dropout keep mask ([E'] x H, 0/1)
        self.attn_keep: Optional[Tensor] = None

    def reset_parameters(self):
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

    def forward(self, x: Tensor, edge_index: Tensor, edge_attr: Optional[Tensor] = None,
                return_attention_weights: bool = False):
        H, C = self.heads, self.out_channels
        x_src = x_dst = self.lin_src(x).view(-1, H, C)
        alpha_src = (x_src * self.att_src).sum(dim=-1)
        alpha_dst = (x_dst * self.att_dst).sum(dim=-1)
        N = x_src.size(0)
        if self.add_self_loops:
            edge_index, edge_attr = remove_self_loops(edge_index, edge_attr)
            edge_index, edge_attr = add_self_loops(edge_index, edge_attr, self.fill_value, N)
        src, dst = edge_index[0], edge_index[1]
        # edge_update(alpha_j, alpha_i, edge_attr, index=dst)
        alpha = alpha_src.index_select(0, src) + alpha_dst.index_select(0, dst)
        if edge_attr is not None and self.lin_edge is not None:
            if edge_attr.dim() == 1:
                edge_attr = edge_attr.view(-1, 1)
            ea = self.lin_edge(edge_attr).view(-1, H, C)
            alpha = alpha + (ea * self.att_edge).sum(dim=-1)
        alpha = F.leaky_relu(alpha, self.negative_slope)
        alpha = pyg_softmax(alpha, dst, N)
        p_att = alpha
        if self.attn_keep is not None and self.training and self.dropout > 0:
            alpha = alpha * self.attn_keep / (1.0 - self.dropout)
        else:
            alpha = F.dropout(alpha, p=self.dropout, training=self.training)
        # propagate: message = alpha.unsqueeze(-1) * x_j ; aggr = 'add'
        msg = alpha.unsqueeze(-1) * x_src.index_select(0, src)
        out = scatter_sum(msg, dst, N)
        if self.concat:
            out = out.view(-1, H * C)
        else:
            out = out.mean(dim=1)
        if self.bias is not None:
            out = out + self.bias
        if return_attention_weights:
            return out, (edge_index, p_att)
        return out


class OracleGATModel(nn.Module):
    """reference utils/models.py:61-152, verbatim layer-stacking rules."""

    def __init__(self, num_node_features, num_edge_features, num_heads, output_node_channels,
                 dim_hidden_layers=[100], dropout_att=0.0, dropout=0.0, activation="relu",
                 concat_heads=False, negative_slope=0.2, standardize=False):
        super().__init__()
        self.dropout = dropout
        self.activation = activation
        self.standardize = standardize
        if self.standardize:
            self.bnorm_node = nn.BatchNorm1d(num_node_features, affine=False)
            self.bnorm_edge = nn.BatchNorm1d(num_edge_features, affine=False)
        kw = dict(heads=num_heads, dropout=dropout_att, edge_dim=num_edge_features,
                  negative_slope=negative_slope)
        if len(dim_hidden_layers) == 1:
            first = [OracleGATConv(num_node_features, dim_hidden_layers[0], concat=False, **kw)]
        else:
            first = [OracleGATConv(num_node_features, dim_hidden_layers[0], concat=concat_heads,
                                   **kw)]
        stacked = []
        for i in range(len(dim_hidden_layers) - 1):
            in_ch = (dim_hidden_layers[i] * num_heads if (concat_heads and num_heads > 1)
                     else dim_hidden_layers[i])
            if i + 1 == len(dim_hidden_layers) - 1:
                stacked.append(OracleGATConv(in_ch, dim_hidden_layers[i + 1], concat=False, **kw))
            else:
                stacked.append(OracleGATConv(in_ch, dim_hidden_layers[i + 1], concat=concat_heads,
                                             **kw))
        self.gat_layers = nn.ModuleList(first + stacked)
        self.linear = nn.Linear(dim_hidden_layers[-1], output_node_channels)
        self.a = {"relu": F.relu, "tanh": F.tanh, "sigmoid": F.sigmoid}[activation]
        # test hook: explicit post-layer dropout keep masks, one [N, out] 0/1
        # tensor per GAT layer (utils/models.py:148 draws them with F.dropout)
        self.post_keep: Optional[list] = None
        # test hook (relu only): the active side of each layer's activation,
        # one [N, out] bool tensor per layer, taken from the product's forward so
        # that a pre-activation within rounding of 0 (where the two sides of the
        # kink give gradients that differ by a whole node's contribution) takes
        # the same branch in both; the pre-activations are kept in act_inputs
        # for the test to check that masks differ only at such points
        self.act_masks: Optional[list] = None
        self.act_inputs: list = []

    def forward(self, data):
        x, edge_index, edge_attr = data.x, data.edge_index, data.edge_attr
        if self.standardize:
            x = self.bnorm_node(x)
            edge_attr = self.bnorm_edge(edge_attr)
        self.act_inputs = []
        for i, l in enumerate(self.gat_layers):
            x = l(x, edge_index, edge_attr)
            if self.act_masks is not None and self.activation == "relu":
                self.act_inputs.append(x.detach())
                x = x * self.act_masks[i].to(x.dtype)
            else:
                x = self.a(x)
            if self.dropout:
                if self.post_keep is not None and self.training:
                    x = x * self.post_keep[i].to(x.dtype) / (1.0 - self.dropout)
                else:
                    x = F.dropout(x, p=self.dropout, training=self.training)
        x = self.linear(x)
        return x.view(-1)
