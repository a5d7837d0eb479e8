"""``torch.ops.sv2n.*``: the C-ABI (include/sv2n.h) registered as PyTorch
operators, with fake (meta) implementations for shape propagation.

This is the operator boundary SURVEY.md §8b names: every kernel group the
fused GAT stack, the output head, the optimizer and the window builder launch
is one ``sv2n::`` op.  The real implementations check shapes / dtypes /
devices, allocate outputs and workspaces from the caching allocator and
launch on the current HIP stream (so every op is capturable into a hipGraph);
the fake implementations return correctly shaped empty tensors, which is what
``torch.compile`` / FakeTensor tracing and ``torch.library.opcheck`` need.

Ops that ACCUMULATE into parameter gradients (``gat_wgrad``,
``prep_bwd_edge``, ``head_bwd``, ``head_mse_bwd``) and the optimizer step
declare those arguments as mutated (``Tensor(a!)``) in their schema.

Reference ops each entry replaces: the comments in include/sv2n.h
(PyG 2.3.0 GATConv pieces, reference utils/models.py:146; GATModel.linear,
utils/models.py:150; Adam, 5_train_SpotV2Net.py:127/:159;
CovarianceLaggedDataset windows, utils/dataset.py:200-282).
"""
from __future__ import annotations

import ctypes
from typing import List, Optional

import torch

from . import _lib

LIB = torch.library.Library("sv2n", "DEF")

_SCHEMAS = {
    "gat_prep": "(Tensor[] W, Tensor[] att_src, Tensor[] att_dst, Tensor[] W_edge, "
                "Tensor[] att_edge, int[] heads, int[] channels, int hl_pad, bool[] need_t, "
                "bool use_edge, bool bf16=False) -> (Tensor[], Tensor[], Tensor[], Tensor)",
    "edge_logits": "(Tensor edge_attr, Tensor wfold, Tensor? edge_index, Tensor canon, "
                   "int num_layers, int heads, int num_graphs, int n, bool planes) -> Tensor[]",
    "project": "(Tensor a, Tensor? planes, Tensor w, bool transpose_w, bool bf16, "
               "Tensor? relu_y=None) -> Tensor",
    "gat_attn_fwd": "(Tensor xs, Tensor? ae, Tensor? rowmask, Tensor? bias, Tensor? keep, "
                    "float keep_scale, int num_graphs, int n, int heads, int channels, "
                    "bool concat, int act, float slope, bool edge_order=False) -> (Tensor, Tensor)",
    "gat_attn_fwd_post": "(Tensor xs, Tensor? ae, Tensor? rowmask, Tensor? bias, Tensor? keep, "
                         "float keep_scale, Tensor post_u, float post_p, int num_graphs, int n, "
                         "int heads, int channels, bool concat, int act, float slope, "
                         "bool edge_order=False) -> (Tensor, Tensor, Tensor)",
    "gat_attn_fwd_head_mse": "(Tensor xs, Tensor? ae, Tensor? rowmask, Tensor? bias, Tensor? keep, "
                             "float keep_scale, Tensor? post_u, float post_p, Tensor head_weight, "
                             "Tensor? head_bias, Tensor target, Tensor(a!)? g_head_weight, "
                             "Tensor(b!)? g_head_bias, int num_graphs, int n, int heads, "
                             "int channels, bool concat, int act, float slope, "
                             "bool edge_order=False, Tensor(c!)? loss_sum=None) "
                             "-> (Tensor, Tensor, Tensor)",
    "project_bf16_export": "(Tensor a, Tensor planes, Tensor w) -> (Tensor, Tensor)",
    "gat_attn_bwd_bf16dx": "(Tensor dy, Tensor y, Tensor xs, Tensor psave, Tensor? keep, "
                           "float keep_scale, Tensor? rowmask, bool with_ae, int num_graphs, "
                           "int n, int heads, int channels, bool concat, int act, float slope, "
                           "bool edge_order=False, Tensor? post_u=None, float post_p=0.0) "
                           "-> (Tensor, Tensor, Tensor)",
    "gat_wgrad_bf16b": "(Tensor x_b, Tensor dxs_b, Tensor W, Tensor att_src, Tensor att_dst, "
                       "Tensor dbias_partial, int heads, int channels, Tensor(a!) gW, "
                       "Tensor(b!)? g_att_src, Tensor(c!)? g_att_dst, Tensor(d!)? g_bias) -> ()",
    "gat_attn_tiled_fwd": "(Tensor xs, Tensor? ae, int num_edges, Tensor? eid, Tensor? rowmask, "
                          "Tensor? bias, Tensor? keep, float keep_scale, int num_graphs, int n, "
                          "int heads, int channels, bool concat, int act, float slope) -> Tensor",
    "gat_attn_fused_fwd": "(Tensor xs, Tensor edge_attr, Tensor wfold, int col0, Tensor? eid, "
                          "Tensor? bias, Tensor? keep, float keep_scale, int num_graphs, int n, "
                          "int heads, int channels, bool concat, int act, float slope, "
                          "bool training) -> (Tensor, Tensor, Tensor)",
    "gat_attn_fused_bwd": "(Tensor dy, Tensor y, Tensor agg, Tensor stats, Tensor xs, "
                          "Tensor edge_attr, Tensor wfold, int col0, Tensor? eid, Tensor? keep, "
                          "float keep_scale, Tensor(a!) dwfold, int num_graphs, int n, int heads, "
                          "int channels, bool concat, int act, float slope) -> (Tensor, Tensor)",
    "gat_attn_bwd": "(Tensor dy, Tensor y, Tensor xs, Tensor psave, Tensor? keep, "
                    "float keep_scale, Tensor? rowmask, bool with_ae, int num_graphs, int n, "
                    "int heads, int channels, bool concat, int act, float slope, "
                    "bool edge_order=False, Tensor? post_u=None, float post_p=0.0) "
                    "-> (Tensor, Tensor, Tensor)",
    "gat_attn_tiled_bwd": "(Tensor dy, Tensor y, Tensor xs, Tensor? ae, int num_edges, "
                          "Tensor? eid, Tensor? keep, float keep_scale, Tensor? rowmask, "
                          "int num_graphs, int n, int heads, int channels, bool concat, int act, "
                          "float slope) -> (Tensor, Tensor, Tensor)",
    "gat_wgrad": "(Tensor? x, Tensor dxs, Tensor W, Tensor att_src, Tensor att_dst, "
                 "Tensor dbias_partial, int heads, int channels, bool bf16, Tensor(a!)? gW, "
                 "Tensor(b!)? g_att_src, Tensor(c!)? g_att_dst, Tensor(d!)? g_bias) -> ()",
    "edge_logits_bwd": "(Tensor edge_attr, Tensor? edge_index, Tensor canon, Tensor[] dae, "
                       "int heads, int num_graphs, int n, int hl_pad, bool planes) -> Tensor",
    "edge_logits_cv": "(Tensor edge_attr, Tensor wfold, Tensor canon, int num_layers, int heads, "
                      "int num_graphs, int n) -> Tensor[]",
    "edge_logits_bwd_cv": "(Tensor edge_attr, Tensor canon, Tensor[] dae, int heads, "
                          "int num_graphs, int n, int hl_pad) -> Tensor",
    "gat_attn_bwd_edge": "(Tensor dy, Tensor y, Tensor xs, Tensor psave, Tensor? keep, "
                         "float keep_scale, Tensor edge_attr, Tensor?[] dae, int layer, "
                         "int hl_pad, int num_graphs, int n, int heads, int channels, "
                         "bool concat, int act, float slope, Tensor? post_u=None, "
                         "float post_p=0.0) -> (Tensor, Tensor, Tensor)",
    "prep_bwd_edge": "(Tensor dwfold, int col0, Tensor W_edge, Tensor att_edge, int heads, "
                     "int channels, Tensor(a!)? gW_edge, Tensor(b!)? g_att_edge) -> ()",
    "prep_bwd_edge_all": "(Tensor dwfold, int[] col0, Tensor[] W_edge, Tensor[] att_edge, "
                         "int[] heads, int[] channels, Tensor(a!)[] gW_edge, "
                         "Tensor(b!)[] g_att_edge) -> ()",
    "head_fwd": "(Tensor x, Tensor weight, Tensor? bias) -> Tensor",
    "head_bwd": "(Tensor x, Tensor weight, Tensor dout, Tensor(a!)? g_weight, "
                "Tensor(b!)? g_bias) -> Tensor",
    "head_mse_fwd": "(Tensor x, Tensor weight, Tensor? bias, Tensor target, "
                    "Tensor(a!)? loss_sum=None) -> (Tensor, Tensor)",
    "head_mse_train": "(Tensor x, Tensor weight, Tensor? bias, Tensor target, "
                      "Tensor(a!)? g_weight, Tensor(b!)? g_bias, Tensor(c!)? loss_sum=None) "
                      "-> (Tensor, Tensor)",
    "head_mse_train_rows": "(Tensor x, Tensor weight, Tensor? bias, Tensor target, "
                           "Tensor(a!) ws) -> Tensor",
    "head_mse_train_reduce": "(Tensor ws, int num_rows, int in_features, int out_features, "
                             "Tensor(a!) loss, Tensor(b!)? g_weight, Tensor(c!)? g_bias, "
                             "Tensor(d!)? loss_sum=None) -> ()",
    "head_mse_bwd": "(Tensor x, Tensor weight, Tensor diff, Tensor grad_loss, "
                    "Tensor(a!)? g_weight, Tensor(b!)? g_bias) -> Tensor",
    "dropout_uniform": "(int rows, int cols, Tensor step, int seed, int salt) -> Tensor",
    "adam_step": "(Tensor(a!) param, Tensor(b!) grad, Tensor(c!) exp_avg, Tensor(d!) exp_avg_sq, "
                 "Tensor(e!) step, Tensor(f!) ticket, float lr, float beta1, float beta2, "
                 "float eps, float weight_decay) -> ()",
    "window_gather": "(Tensor vol, Tensor volvol, Tensor starts, int seq_length, "
                     "int future_steps, Tensor canon, Tensor(a!) x, Tensor(b!) edge_attr, "
                     "Tensor(c!) y, int start_offset=0, Tensor? diag=None, "
                     "Tensor(d!)? x_bf16=None, bool cov_var_only=False, bool skip_x=False) -> ()",
    "project_a16": "(Tensor a_bf16, int k, Tensor planes, Tensor w) -> Tensor",
}
for _name, _schema in _SCHEMAS.items():
    LIB.define(_name + _schema)


def _impl(name):
    def deco(fn):
        LIB.impl(name, fn, "CUDA")
        return fn
    return deco


def _fake(name):
    return torch.library.register_fake("sv2n::" + name)


def _p(t: Optional[torch.Tensor]):
    return None if t is None or t.numel() == 0 else t.data_ptr()


def _st(t: torch.Tensor) -> int:
    return _lib.stream_handle(t.device)


def _need(cond: bool, msg: str) -> None:
    if not cond:
        raise RuntimeError("sv2n: " + msg)


def _f32(*ts) -> None:
    for t in ts:
        if t is not None:
            _need(t.dtype == torch.float32, f"expected float32, got {t.dtype}")
            _need(t.is_cuda, "expected a ROCm device tensor")


def _dense(*ts) -> None:
    """The kernels address these through raw pointers as dense row-major
    buffers: refuse anything else (an error, never a wrong read)."""
    for t in ts:
        if t is not None and t.numel() > 0:
            _need(t.is_contiguous(), f"expected a contiguous tensor of shape {tuple(t.shape)}")
            _need(t.is_cuda, "expected a ROCm device tensor")


def _rows(xs: torch.Tensor, rows: int, min_cols: int, what: str) -> None:
    _need(xs.dim() == 2 and xs.shape[0] == rows and xs.shape[1] >= min_cols and
          xs.stride(1) == 1 and xs.stride(0) >= xs.shape[1], f"{what}: expected [{rows}, >= "
          f"{min_cols}] rows with unit column stride, got {tuple(xs.shape)} / {xs.stride()}")


def _ldx(H: int, C: int) -> int:
    return (H * C + 2 * H + 3) // 4 * 4


# --------------------------------------------------------------------------
# weight preparation (sv2n_gat_prep_fwd_all)
# --------------------------------------------------------------------------
def _prep_shapes(W, heads, channels, need_t, kpad, np=3):
    out = []
    for l, w in enumerate(W):
        F = w.shape[1]
        ldx = _ldx(heads[l], channels[l])
        out.append(((ldx, F), (np, ldx, kpad(F)), (np, F, kpad(ldx)) if need_t[l] else (0,)))
    return out


def _waug_placeholder(w: torch.Tensor, shape) -> torch.Tensor:
    """Waug's shape without its data (bf16-mode gat_prep): consumers read only
    the shape; ops.project / weight_planes refuse it (ops._has_data).  One
    uninitialised element, expanded: no fill launch (new_zeros launched a
    4.6 µs fill kernel in every captured C3 step)."""
    return w.new_empty(1).expand(shape)


def _kpad(K: int) -> int:
    return (K + 63) // 64 * 64  # sv2n_split3_kpad


@_impl("gat_prep")
def _gat_prep(W, att_src, att_dst, W_edge, att_edge, heads, channels, hl_pad, need_t, use_edge,
              bf16=False):
    lib = _lib.load()
    L = len(W)
    _f32(*W, *att_src, *att_dst, *W_edge, *att_edge)
    dev = W[0].device
    D = W_edge[0].shape[1] if use_edge else 0
    wf = torch.empty(D, hl_pad, device=dev) if use_edge else torch.empty(0, device=dev)
    arr = (_lib.PrepLayer * L)()
    waugs, planes, planes_t = [], [], []
    np = 1 if bf16 else 3
    for l, (s_w, s_p, s_t) in enumerate(_prep_shapes(W, heads, channels, need_t, _kpad, np)):
        # bf16 mode: every GEMM takes the planes, so Waug itself is not
        # written (ABI 19) and stands as a stride-0 placeholder of its shape
        waug = _waug_placeholder(W[l], s_w) if bf16 else torch.empty(s_w, device=dev)
        pl = torch.empty(s_p, device=dev, dtype=torch.int16)
        plt = torch.empty(s_t, device=dev, dtype=torch.int16)
        arr[l] = _lib.PrepLayer(
            W[l].data_ptr(), att_src[l].data_ptr(), att_dst[l].data_ptr(), heads[l], channels[l],
            W[l].shape[1], s_w[0], None if bf16 else waug.data_ptr(), pl.data_ptr(), _p(plt),
            W_edge[l].data_ptr() if use_edge else None,
            att_edge[l].data_ptr() if use_edge else None, D, hl_pad, l * heads[0],
            _p(wf) if use_edge else None, np)
        waugs.append(waug)
        planes.append(pl)
        planes_t.append(plt)
    _lib.check(lib.sv2n_gat_prep_fwd_all(ctypes.addressof(arr), L, _st(W[0])),
               "sv2n_gat_prep_fwd_all")
    return waugs, planes, planes_t, wf


@_fake("gat_prep")
def _gat_prep_fake(W, att_src, att_dst, W_edge, att_edge, heads, channels, hl_pad, need_t,
                   use_edge, bf16=False):
    D = W_edge[0].shape[1] if use_edge else 0
    w0 = W[0]
    shp = _prep_shapes(W, heads, channels, need_t, _kpad, 1 if bf16 else 3)
    return ([_waug_placeholder(w0, a) if bf16 else w0.new_empty(a) for a, _, _ in shp],
            [w0.new_empty(b, dtype=torch.int16) for _, b, _ in shp],
            [w0.new_empty(c, dtype=torch.int16) for _, _, c in shp],
            w0.new_empty((D, hl_pad) if use_edge else (0,)))


# --------------------------------------------------------------------------
# edge logits (sv2n_edge_logits_fwd / _planes) and their weight gradient
# --------------------------------------------------------------------------
def _ae_shape(planes, E, num_graphs, n, heads, edge_index):
    """[H][E] planes (tiled path); edge order [E][H] for a canonical batch
    (edge_index None, n > 1); else the dense per-graph [B][n][n][H] block."""
    if planes:
        return (heads, E)
    return (E, heads) if edge_order(edge_index, n) else (num_graphs, n, n, heads)


def edge_order(edge_index, n: int) -> bool:
    """Whether sv2n_edge_logits_fwd writes (and the attention kernels take)
    the edge-ordered AE layout: canonical batches of complete graphs."""
    return edge_index is None and n > 1


@_impl("edge_logits")
def _edge_logits(edge_attr, wfold, edge_index, canon, num_layers, heads, num_graphs, n, planes):
    lib = _lib.load()
    _f32(edge_attr, wfold)
    _dense(edge_attr, wfold, edge_index, canon)
    E, D = edge_attr.shape
    _need(wfold.shape[0] == D and num_layers * heads <= wfold.shape[1], "wfold shape")
    _need(edge_index is None or tuple(edge_index.shape) == (2, E), "edge_index shape")
    _need(canon.numel() == n * (n - 1), "canonical table shape")
    _need(planes or edge_index is not None or E == num_graphs * n * (n - 1),
          "canonical batch edge count")
    outs = [torch.empty(_ae_shape(planes, E, num_graphs, n, heads, edge_index),
                        device=edge_attr.device)
            for _ in range(num_layers)]
    if E == 0:
        return outs
    _need(edge_attr.is_contiguous() and edge_attr.data_ptr() % 16 == 0, "edge_attr alignment")
    ptrs = _lib.ptr_array([o.data_ptr() for o in outs])
    hp = wfold.shape[1]
    if planes:
        rc = lib.sv2n_edge_logits_fwd_planes(edge_attr.data_ptr(), E, D, wfold.data_ptr(), hp,
                                             ptrs, num_layers, heads, _st(edge_attr))
    else:
        rc = lib.sv2n_edge_logits_fwd(edge_attr.data_ptr(), E, D, _p(edge_index),
                                      canon.data_ptr(), wfold.data_ptr(), hp, ptrs, num_layers,
                                      heads, num_graphs, n, _st(edge_attr))
    _lib.check(rc, "sv2n_edge_logits_fwd")
    return outs


@_fake("edge_logits")
def _edge_logits_fake(edge_attr, wfold, edge_index, canon, num_layers, heads, num_graphs, n,
                      planes):
    E = edge_attr.shape[0]
    return [edge_attr.new_empty(_ae_shape(planes, E, num_graphs, n, heads, edge_index))
            for _ in range(num_layers)]


@_impl("edge_logits_bwd")
def _edge_logits_bwd(edge_attr, edge_index, canon, dae, heads, num_graphs, n, hl_pad, planes):
    lib = _lib.load()
    _dense(edge_attr, edge_index, canon, *dae)
    E, D = edge_attr.shape
    dev = edge_attr.device
    L = len(dae)
    for d in dae:
        _need(d.numel() == (heads * E if planes or edge_order(edge_index, n)
                            else num_graphs * n * n * heads), "dae shape")
    ptrs = _lib.ptr_array([d.data_ptr() for d in dae])
    ws_n = lib.sv2n_edge_logits_bwd_workspace(D, hl_pad)
    ws = torch.empty(ws_n, device=dev)
    dwf = torch.empty(D, hl_pad, device=dev)
    if planes:
        rc = lib.sv2n_edge_logits_bwd_planes(edge_attr.data_ptr(), E, D, _p(edge_index), ptrs, L,
                                             heads, ws.data_ptr(), ws_n, dwf.data_ptr(), hl_pad,
                                             _st(edge_attr))
    else:
        rc = lib.sv2n_edge_logits_bwd(edge_attr.data_ptr(), E, D, _p(edge_index),
                                      canon.data_ptr(), ptrs, L, heads, num_graphs, n,
                                      ws.data_ptr(), ws_n, dwf.data_ptr(), hl_pad, _st(edge_attr))
    _lib.check(rc, "sv2n_edge_logits_bwd")
    return dwf


@_fake("edge_logits_bwd")
def _edge_logits_bwd_fake(edge_attr, edge_index, canon, dae, heads, num_graphs, n, hl_pad,
                          planes):
    return edge_attr.new_empty((edge_attr.shape[1], hl_pad))


def _cv_common(edge_attr, canon, num_graphs, n):
    _dense(edge_attr, canon)
    E, D = edge_attr.shape
    _need(D % 3 == 0, "covariance-layout edge_attr has 3 x seq_length columns")
    _need(E == num_graphs * n * (n - 1), "covariance layout: canonical complete graphs")
    _need(canon.numel() == n * (n - 1), "canonical table shape")
    return E, D


@_impl("edge_logits_cv")
def _edge_logits_cv(edge_attr, wfold, canon, num_layers, heads, num_graphs, n):
    """sv2n_edge_logits_fwd_cv: edge_logits for edge features in the
    reference's covariance layout (the caller vouches for it)."""
    lib = _lib.load()
    _f32(edge_attr, wfold)
    E, D = _cv_common(edge_attr, canon, num_graphs, n)
    _dense(wfold)
    _need(wfold.shape[0] == D and num_layers * heads <= wfold.shape[1], "wfold shape")
    outs = [torch.empty(E, heads, device=edge_attr.device) for _ in range(num_layers)]
    if E == 0:
        return outs
    ptrs = _lib.ptr_array([o.data_ptr() for o in outs])
    _lib.check(lib.sv2n_edge_logits_fwd_cv(edge_attr.data_ptr(), num_graphs, n, D // 3,
                                           canon.data_ptr(), wfold.data_ptr(), wfold.shape[1],
                                           ptrs, num_layers, heads, _st(edge_attr)),
               "sv2n_edge_logits_fwd_cv")
    return outs


@_fake("edge_logits_cv")
def _edge_logits_cv_fake(edge_attr, wfold, canon, num_layers, heads, num_graphs, n):
    return [edge_attr.new_empty((edge_attr.shape[0], heads)) for _ in range(num_layers)]


@_impl("edge_logits_bwd_cv")
def _edge_logits_bwd_cv(edge_attr, canon, dae, heads, num_graphs, n, hl_pad):
    lib = _lib.load()
    _f32(edge_attr, *dae)
    E, D = _cv_common(edge_attr, canon, num_graphs, n)
    _dense(*dae)
    for d in dae:
        _need(d.numel() == heads * E, "dae shape")
    dev = edge_attr.device
    dwf = torch.empty(D, hl_pad, device=dev)
    if E == 0:
        return dwf.zero_()
    ptrs = _lib.ptr_array([d.data_ptr() for d in dae])
    ws_n = lib.sv2n_edge_logits_bwd_cv_workspace(D // 3, hl_pad)
    ws = torch.empty(ws_n, device=dev)
    _lib.check(lib.sv2n_edge_logits_bwd_cv(edge_attr.data_ptr(), num_graphs, n, D // 3,
                                           canon.data_ptr(), ptrs, len(dae), heads, ws.data_ptr(),
                                           ws_n, dwf.data_ptr(), hl_pad, _st(edge_attr)),
               "sv2n_edge_logits_bwd_cv")
    return dwf


@_fake("edge_logits_bwd_cv")
def _edge_logits_bwd_cv_fake(edge_attr, canon, dae, heads, num_graphs, n, hl_pad):
    return edge_attr.new_empty((edge_attr.shape[1], hl_pad))


@_impl("prep_bwd_edge")
def _prep_bwd_edge(dwfold, col0, W_edge, att_edge, heads, channels, gW_edge, g_att_edge):
    lib = _lib.load()
    _lib.check(lib.sv2n_gat_prep_bwd_edge(dwfold.data_ptr(), dwfold.shape[1], col0,
                                          W_edge.data_ptr(), att_edge.data_ptr(), heads, channels,
                                          W_edge.shape[1], _p(gW_edge), _p(g_att_edge),
                                          _st(dwfold)), "sv2n_gat_prep_bwd_edge")


@_fake("prep_bwd_edge")
def _prep_bwd_edge_fake(dwfold, col0, W_edge, att_edge, heads, channels, gW_edge, g_att_edge):
    return None


@_impl("prep_bwd_edge_all")
def _prep_bwd_edge_all(dwfold, col0, W_edge, att_edge, heads, channels, gW_edge, g_att_edge):
    """prep_bwd_edge of every layer in one launch (sv2n_gat_prep_bwd_edge_all)."""
    lib = _lib.load()
    L = len(W_edge)
    arr = (_lib.EdgeGradLayer * L)()
    for l in range(L):
        arr[l] = _lib.EdgeGradLayer(W_edge[l].data_ptr(), att_edge[l].data_ptr(),
                                    gW_edge[l].data_ptr(), g_att_edge[l].data_ptr(), heads[l],
                                    channels[l], col0[l])
    _lib.check(lib.sv2n_gat_prep_bwd_edge_all(dwfold.data_ptr(), dwfold.shape[1],
                                              W_edge[0].shape[1], arr, L, _st(dwfold)),
               "sv2n_gat_prep_bwd_edge_all")


@_fake("prep_bwd_edge_all")
def _prep_bwd_edge_all_fake(dwfold, col0, W_edge, att_edge, heads, channels, gW_edge, g_att_edge):
    return None


# --------------------------------------------------------------------------
# projection GEMMs (sv2n_gemm_f32x3 / sv2n_gemm_bf16 / sv2n_gemm_f32)
# --------------------------------------------------------------------------
@_impl("project")
def _project(a, planes, w, transpose_w, bf16, relu_y=None):
    """relu_y: the consumer's ReLU backward fused into the store, out = (relu_y
    > 0) ? a·w : 0 (sv2n_gemm_f32x3_relu; f32 planes path only)."""
    from .ops import project_planes
    _f32(a, w, relu_y)
    return project_planes(a, planes, w, transpose_w, bf16, relu_y)


@_fake("project")
def _project_fake(a, planes, w, transpose_w, bf16, relu_y=None):
    N = w.shape[1] if transpose_w else w.shape[0]
    return a.new_empty((a.shape[0], N))


def _pad_to(k: int, m: int) -> int:
    return (k + m - 1) // m * m


@_impl("project_bf16_export")
def _project_bf16_export(a, planes, w):
    """The bf16-mode projection a·wᵀ (sv2n_gemm_bf16) that also returns bf16(a)
    [M][round_up(K, 64)] (zero past K), written by the GEMM's own operand
    staging (sv2n_gemm_bf16_export): the layer's weight-gradient operand."""
    lib = _lib.load()
    _f32(a, w)
    M, K = a.shape
    N = w.shape[0]
    _need(a.stride(1) == 1 and a.stride(0) % 4 == 0 and a.data_ptr() % 16 == 0,
          "a: 16-B aligned rows")
    out = torch.empty(M, N, device=a.device, dtype=torch.float32)
    ab = torch.empty(M, _pad_to(K, 64), device=a.device, dtype=torch.bfloat16)
    _lib.check(lib.sv2n_gemm_bf16_export(a.data_ptr(), a.stride(0), planes.data_ptr(),
                                         out.data_ptr(), out.stride(0), M, N, K, ab.data_ptr(),
                                         ab.stride(0), _st(a)), "sv2n_gemm_bf16_export")
    return out, ab


@_fake("project_bf16_export")
def _project_bf16_export_fake(a, planes, w):
    return (a.new_empty((a.shape[0], w.shape[0])),
            a.new_empty((a.shape[0], _pad_to(a.shape[1], 64)), dtype=torch.bfloat16))


# --------------------------------------------------------------------------
# fused attention (sv2n_gat_attn_* and the tiled forms)
# --------------------------------------------------------------------------
def _oc(heads, channels, concat):
    return heads * channels if concat else channels


def _attn_fwd(xs, ae, rowmask, bias, keep, keep_scale, post_u, post_p, num_graphs, n, heads,
              channels, concat, act, slope, edge_order):
    lib = _lib.load()
    _f32(xs, ae, bias, post_u)
    N, OC = num_graphs * n, _oc(heads, channels, concat)
    _rows(xs, N, heads * channels + 2 * heads, "xs")
    _dense(ae, rowmask, bias, keep, post_u)
    _need(ae is None or ae.numel() == num_graphs * n * (n - int(edge_order)) * heads, "ae shape")
    _need(not edge_order or rowmask is None, "edge-ordered ae needs complete graphs")
    _need(bias is None or bias.numel() == OC, "bias shape")
    _need(keep is None or keep.numel() == num_graphs * heads * 1024, "keep shape")
    _need(rowmask is None or rowmask.numel() >= N, "rowmask shape")
    _need(post_u is None or (post_u.numel() == N * OC and 0.0 <= post_p < 1.0), "post_u / post_p")
    y = torch.empty(N, OC, device=xs.device)
    ps = torch.empty(num_graphs, heads, 32, 32, device=xs.device)
    out = torch.empty(N, OC, device=xs.device) if post_u is not None else None
    _lib.check(lib.sv2n_gat_attn_fwd(xs.data_ptr(), xs.stride(0), _p(ae), int(edge_order),
                                     _p(rowmask), _p(bias),
                                     _p(keep), keep_scale, y.data_ptr(), ps.data_ptr(),
                                     _p(post_u), post_p, _p(out),
                                     num_graphs, n, heads, channels, int(concat), act, slope,
                                     _st(xs)), "sv2n_gat_attn_fwd")
    return y, ps, out


@_impl("gat_attn_fwd")
def _gat_attn_fwd(xs, ae, rowmask, bias, keep, keep_scale, num_graphs, n, heads, channels,
                  concat, act, slope, edge_order=False):
    y, ps, _ = _attn_fwd(xs, ae, rowmask, bias, keep, keep_scale, None, 0.0, num_graphs, n, heads,
                         channels, concat, act, slope, edge_order)
    return y, ps


@_fake("gat_attn_fwd")
def _gat_attn_fwd_fake(xs, ae, rowmask, bias, keep, keep_scale, num_graphs, n, heads, channels,
                       concat, act, slope, edge_order=False):
    return (xs.new_empty((num_graphs * n, _oc(heads, channels, concat))),
            xs.new_empty((num_graphs, heads, 32, 32)))


@_impl("gat_attn_fwd_post")
def _gat_attn_fwd_post(xs, ae, rowmask, bias, keep, keep_scale, post_u, post_p, num_graphs, n,
                       heads, channels, concat, act, slope, edge_order=False):
    """gat_attn_fwd with GATModel's post-layer dropout fused into the store
    (utils/models.py:148): also returns out = y · (post_u >= post_p) / (1 - post_p)."""
    return _attn_fwd(xs, ae, rowmask, bias, keep, keep_scale, post_u, post_p, num_graphs, n,
                     heads, channels, concat, act, slope, edge_order)


@_fake("gat_attn_fwd_post")
def _gat_attn_fwd_post_fake(xs, ae, rowmask, bias, keep, keep_scale, post_u, post_p, num_graphs,
                            n, heads, channels, concat, act, slope, edge_order=False):
    oc = _oc(heads, channels, concat)
    return (xs.new_empty((num_graphs * n, oc)), xs.new_empty((num_graphs, heads, 32, 32)),
            xs.new_empty((num_graphs * n, oc)))


def attn_fwd_head_mse_supported(num_graphs: int, n: int, heads: int, channels: int,
                                concat: bool) -> bool:
    """Whether sv2n_gat_attn_fwd_head_mse runs this layer shape (include/sv2n.h)."""
    return bool(_lib.load().sv2n_gat_attn_fwd_head_mse_supported(num_graphs, n, heads, channels,
                                                                 int(concat)))


@_impl("gat_attn_fwd_head_mse")
def _gat_attn_fwd_head_mse(xs, ae, rowmask, bias, keep, keep_scale, post_u, post_p, head_weight,
                           head_bias, target, g_head_weight, g_head_bias, num_graphs, n, heads,
                           channels, concat, act, slope, edge_order=False, loss_sum=None):
    """The last layer's attention with GATModel.linear (out_features 1) and the
    MSE loss fused in: returns (dz, psave, loss) — dz the gradient the layer's
    backward starts from (identity activation, no post dropout) — and
    accumulates the head's parameter gradients."""
    lib = _lib.load()
    _f32(xs, ae, bias, post_u, head_weight, head_bias, target)
    N, OC = num_graphs * n, _oc(heads, channels, concat)
    _rows(xs, N, heads * channels + 2 * heads, "xs")
    _dense(ae, rowmask, bias, keep, post_u, head_weight, head_bias, target, g_head_weight,
           g_head_bias)
    _need(ae is None or ae.numel() == num_graphs * n * (n - int(edge_order)) * heads, "ae shape")
    _need(not edge_order or rowmask is None, "edge-ordered ae needs complete graphs")
    _need(bias is None or bias.numel() == OC, "bias shape")
    _need(keep is None or keep.numel() == num_graphs * heads * 1024, "keep shape")
    _need(rowmask is None or rowmask.numel() >= N, "rowmask shape")
    _need(post_u is None or (post_u.numel() == N * OC and 0.0 <= post_p < 1.0), "post_u / post_p")
    _need(head_weight.numel() == OC and (head_bias is None or head_bias.numel() == 1),
          "head shape (out_features 1)")
    _need(target.numel() == N, f"target has {target.numel()} elements, expected {N}")
    dz = torch.empty(N, OC, device=xs.device)
    ps = torch.empty(num_graphs, heads, 32, 32, device=xs.device)
    loss = torch.empty((), device=xs.device)
    _need(loss_sum is None or (loss_sum.numel() == 1 and loss_sum.dtype == torch.float32),
          "loss_sum: one float32")
    ws_n = lib.sv2n_gat_attn_fwd_head_mse_workspace(num_graphs, heads, channels, int(concat))
    ws = torch.empty(ws_n, device=xs.device)
    _lib.check(lib.sv2n_gat_attn_fwd_head_mse(
        xs.data_ptr(), xs.stride(0), _p(ae), int(edge_order), _p(rowmask), _p(bias), _p(keep),
        keep_scale, dz.data_ptr(), ps.data_ptr(), _p(post_u), post_p, head_weight.data_ptr(),
        _p(head_bias), target.data_ptr(), loss.data_ptr(), _p(loss_sum), _p(g_head_weight),
        _p(g_head_bias), ws.data_ptr(), ws_n, num_graphs, n, heads, channels, int(concat), act,
        slope, _st(xs)), "sv2n_gat_attn_fwd_head_mse")
    return dz, ps, loss


@_fake("gat_attn_fwd_head_mse")
def _gat_attn_fwd_head_mse_fake(xs, ae, rowmask, bias, keep, keep_scale, post_u, post_p,
                                head_weight, head_bias, target, g_head_weight, g_head_bias,
                                num_graphs, n, heads, channels, concat, act, slope,
                                edge_order=False, loss_sum=None):
    return (xs.new_empty((num_graphs * n, _oc(heads, channels, concat))),
            xs.new_empty((num_graphs, heads, 32, 32)), xs.new_empty(()))


@_impl("gat_attn_tiled_fwd")
def _gat_attn_tiled_fwd(xs, ae, num_edges, eid, rowmask, bias, keep, keep_scale, num_graphs, n,
                        heads, channels, concat, act, slope):
    lib = _lib.load()
    _f32(xs, ae, bias)
    N = num_graphs * n
    _rows(xs, N, heads * channels + 2 * heads, "xs")
    _dense(ae, eid, rowmask, bias, keep)
    _need(ae is None or ae.numel() == heads * num_edges, "ae shape")
    _need(eid is None or eid.numel() == N * n, "eid shape")
    _need(bias is None or bias.numel() == _oc(heads, channels, concat), "bias shape")
    _need(keep is None or keep.numel() == num_graphs * heads * n * n, "keep shape")
    y = torch.empty(N, _oc(heads, channels, concat), device=xs.device)
    ws_n = lib.sv2n_gat_attn_tiled_workspace(num_graphs, n, heads, channels, int(concat))
    ws = torch.empty(max(ws_n, 1), device=xs.device)
    _lib.check(lib.sv2n_gat_attn_tiled_fwd(
        xs.data_ptr(), xs.stride(0), _p(ae), num_edges, _p(eid), _p(rowmask), _p(bias), _p(keep),
        keep_scale, y.data_ptr(), ws.data_ptr(), ws_n, num_graphs, n, heads, channels,
        int(concat), act, slope, _st(xs)), "sv2n_gat_attn_tiled_fwd")
    return y


@_fake("gat_attn_tiled_fwd")
def _gat_attn_tiled_fwd_fake(xs, ae, num_edges, eid, rowmask, bias, keep, keep_scale, num_graphs,
                             n, heads, channels, concat, act, slope):
    return xs.new_empty((num_graphs * n, _oc(heads, channels, concat)))


def fused_supported(n: int, heads: int, channels: int, edge_dim: int) -> bool:
    """Whether sv2n_gat_attn_fused_* take this layer shape (include/sv2n.h)."""
    return bool(_lib.load().sv2n_gat_attn_fused_supported(n, heads, channels, edge_dim))


def _fused_common(xs, edge_attr, wfold, col0, eid, num_graphs, n, heads, channels):
    N = num_graphs * n
    _rows(xs, N, heads * channels + 2 * heads, "xs")
    _need(xs.stride(0) % 4 == 0 and xs.data_ptr() % 16 == 0, "xs: 16-B aligned rows needed")
    _dense(edge_attr, wfold, eid)
    _need(edge_attr.dim() == 2, "edge_attr must be [E, D]")
    _need(wfold.dim() == 2 and wfold.shape[0] == edge_attr.shape[1] and
          0 <= col0 and col0 + heads <= wfold.shape[1], "wfold / col0 shape")
    if eid is None:
        _need(edge_attr.shape[0] == N * (n - 1), "canonical edge_attr needs num_graphs*n*(n-1) rows")
        _need(edge_attr.data_ptr() % 16 == 0, "edge_attr must be 16-B aligned")
    else:
        _need(eid.numel() == N * n and eid.dtype == torch.int32, "eid shape")
    _need(fused_supported(n, heads, channels, edge_attr.shape[1]), "unsupported fused shape")


@_impl("gat_attn_fused_fwd")
def _gat_attn_fused_fwd(xs, edge_attr, wfold, col0, eid, bias, keep, keep_scale, num_graphs, n,
                        heads, channels, concat, act, slope, training):
    lib = _lib.load()
    _f32(xs, edge_attr, wfold, bias)
    _fused_common(xs, edge_attr, wfold, col0, eid, num_graphs, n, heads, channels)
    _dense(bias, keep)
    N = num_graphs * n
    _need(bias is None or bias.numel() == _oc(heads, channels, concat), "bias shape")
    _need(keep is None or keep.numel() == num_graphs * heads * n * n, "keep shape")
    dev = xs.device
    y = torch.empty(N, _oc(heads, channels, concat), device=dev)
    agg = torch.empty(N, heads * channels, device=dev) if training else torch.empty(0, device=dev)
    stats = torch.empty(N, 4 * heads, device=dev) if training else torch.empty(0, device=dev)
    _lib.check(lib.sv2n_gat_attn_fused_fwd(
        xs.data_ptr(), xs.stride(0), edge_attr.data_ptr(), edge_attr.shape[1], wfold.data_ptr(),
        wfold.shape[1], col0, _p(eid), _p(bias), _p(keep), keep_scale, y.data_ptr(), _p(agg),
        _p(stats), num_graphs, n, heads, channels, int(concat), act, slope, _st(xs)),
        "sv2n_gat_attn_fused_fwd")
    return y, agg, stats


@_fake("gat_attn_fused_fwd")
def _gat_attn_fused_fwd_fake(xs, edge_attr, wfold, col0, eid, bias, keep, keep_scale, num_graphs,
                             n, heads, channels, concat, act, slope, training):
    N = num_graphs * n
    return (xs.new_empty((N, _oc(heads, channels, concat))),
            xs.new_empty((N, heads * channels) if training else (0,)),
            xs.new_empty((N, 4 * heads) if training else (0,)))


@_impl("gat_attn_fused_bwd")
def _gat_attn_fused_bwd(dy, y, agg, stats, xs, edge_attr, wfold, col0, eid, keep, keep_scale,
                        dwfold, num_graphs, n, heads, channels, concat, act, slope):
    lib = _lib.load()
    _f32(dy, y, agg, stats, xs, edge_attr, wfold, dwfold)
    _fused_common(xs, edge_attr, wfold, col0, eid, num_graphs, n, heads, channels)
    N, OC = num_graphs * n, _oc(heads, channels, concat)
    _dense(dy, y, agg, stats, keep, dwfold)
    _need(dy.numel() == N * OC and y.numel() == N * OC, "dy / y shape")
    _need(agg.numel() == N * heads * channels and stats.numel() == N * 4 * heads,
          "agg / stats: pass the training forward's outputs")
    _need(keep is None or keep.numel() == num_graphs * heads * n * n, "keep shape")
    _need(dwfold.shape == wfold.shape, "dwfold shape")
    dev = xs.device
    dxs = torch.empty_like(xs)
    dbp = torch.empty(num_graphs * ((n + 31) // 32), OC, device=dev)
    ws_n = lib.sv2n_gat_attn_fused_bwd_workspace(num_graphs, n, heads, channels,
                                                 edge_attr.shape[1])
    ws = torch.empty(ws_n, device=dev)
    _lib.check(lib.sv2n_gat_attn_fused_bwd(
        dy.data_ptr(), y.data_ptr(), agg.data_ptr(), stats.data_ptr(), xs.data_ptr(),
        xs.stride(0), edge_attr.data_ptr(), edge_attr.shape[1], wfold.data_ptr(),
        wfold.shape[1], col0, _p(eid), _p(keep), keep_scale, dxs.data_ptr(), dbp.data_ptr(),
        dwfold.data_ptr(), ws.data_ptr(), ws_n, num_graphs, n, heads, channels, int(concat), act,
        slope, _st(xs)), "sv2n_gat_attn_fused_bwd")
    return dxs, dbp


@_fake("gat_attn_fused_bwd")
def _gat_attn_fused_bwd_fake(dy, y, agg, stats, xs, edge_attr, wfold, col0, eid, keep,
                             keep_scale, dwfold, num_graphs, n, heads, channels, concat, act,
                             slope):
    return (torch.empty_like(xs),
            xs.new_empty((num_graphs * ((n + 31) // 32), _oc(heads, channels, concat))))


def _dae_shape(edge_order, num_graphs, n, heads):
    return (num_graphs * n * (n - 1), heads) if edge_order else (num_graphs, n, n, heads)


@_impl("gat_attn_bwd")
def _gat_attn_bwd(dy, y, xs, psave, keep, keep_scale, rowmask, with_ae, num_graphs, n, heads,
                  channels, concat, act, slope, edge_order=False, post_u=None, post_p=0.0):
    lib = _lib.load()
    _f32(dy, y, xs, psave, post_u)
    N, OC = num_graphs * n, _oc(heads, channels, concat)
    _rows(xs, N, heads * channels + 2 * heads, "xs")
    _dense(dy, y, psave, keep, rowmask, post_u)
    _need(dy.numel() == N * OC and y.numel() == N * OC, "dy / y shape")
    _need(post_u is None or (post_u.numel() == N * OC and 0.0 <= post_p < 1.0), "post_u / post_p")
    _need(psave.numel() == num_graphs * heads * 1024, "psave shape")
    _need(keep is None or keep.numel() == num_graphs * heads * 1024, "keep shape")
    dev = xs.device
    dxs = torch.empty_like(xs)
    _need(not edge_order or rowmask is None, "edge-ordered ae needs complete graphs")
    dae = torch.empty(_dae_shape(edge_order, num_graphs, n, heads), device=dev) if with_ae else \
        torch.empty(0, device=dev)
    dbp = torch.empty(num_graphs, _oc(heads, channels, concat), device=dev)
    _lib.check(lib.sv2n_gat_attn_bwd(dy.data_ptr(), y.data_ptr(), xs.data_ptr(), xs.stride(0),
                                     psave.data_ptr(), _p(keep), keep_scale, _p(post_u), post_p,
                                     _p(rowmask), dxs.data_ptr(), _p(dae), int(edge_order),
                                     dbp.data_ptr(),
                                     num_graphs, n,
                                     heads, channels, int(concat), act, slope, _st(xs)),
               "sv2n_gat_attn_bwd")
    return dxs, dae, dbp


@_fake("gat_attn_bwd")
def _gat_attn_bwd_fake(dy, y, xs, psave, keep, keep_scale, rowmask, with_ae, num_graphs, n,
                       heads, channels, concat, act, slope, edge_order=False, post_u=None,
                       post_p=0.0):
    return (torch.empty_like(xs),
            xs.new_empty(_dae_shape(edge_order, num_graphs, n, heads) if with_ae else (0,)),
            xs.new_empty((num_graphs, _oc(heads, channels, concat))))


@_impl("gat_attn_bwd_bf16dx")
def _gat_attn_bwd_bf16dx(dy, y, xs, psave, keep, keep_scale, rowmask, with_ae, num_graphs, n,
                         heads, channels, concat, act, slope, edge_order=False, post_u=None,
                         post_p=0.0):
    """gat_attn_bwd returning dxs as bf16 [N][round_up(ldx, 8)] (columns past
    ldx zero; sv2n_gat_attn_bwd_bf16dx): the bf16 weight-gradient operand."""
    lib = _lib.load()
    _f32(dy, y, xs, psave, post_u)
    N, OC = num_graphs * n, _oc(heads, channels, concat)
    _rows(xs, N, heads * channels + 2 * heads, "xs")
    _dense(dy, y, psave, keep, rowmask, post_u)
    _need(dy.numel() == N * OC and y.numel() == N * OC, "dy / y shape")
    _need(post_u is None or (post_u.numel() == N * OC and 0.0 <= post_p < 1.0), "post_u / post_p")
    _need(psave.numel() == num_graphs * heads * 1024, "psave shape")
    _need(keep is None or keep.numel() == num_graphs * heads * 1024, "keep shape")
    _need(not edge_order or rowmask is None, "edge-ordered ae needs complete graphs")
    dev = xs.device
    ldx = xs.stride(0)
    dxb = torch.empty(N, _pad_to(ldx, 8), device=dev, dtype=torch.bfloat16)
    dae = torch.empty(_dae_shape(edge_order, num_graphs, n, heads), device=dev) if with_ae else \
        torch.empty(0, device=dev)
    dbp = torch.empty(num_graphs, OC, device=dev)
    _lib.check(lib.sv2n_gat_attn_bwd_bf16dx(
        dy.data_ptr(), y.data_ptr(), xs.data_ptr(), ldx, psave.data_ptr(), _p(keep), keep_scale,
        _p(post_u), post_p, _p(rowmask), dxb.data_ptr(), dxb.stride(0), _p(dae), int(edge_order),
        dbp.data_ptr(), num_graphs, n, heads, channels, int(concat), act, slope, _st(xs)),
        "sv2n_gat_attn_bwd_bf16dx")
    return dxb, dae, dbp


@_fake("gat_attn_bwd_bf16dx")
def _gat_attn_bwd_bf16dx_fake(dy, y, xs, psave, keep, keep_scale, rowmask, with_ae, num_graphs,
                              n, heads, channels, concat, act, slope, edge_order=False,
                              post_u=None, post_p=0.0):
    return (xs.new_empty((xs.shape[0], _pad_to(xs.stride(0), 8)), dtype=torch.bfloat16),
            xs.new_empty(_dae_shape(edge_order, num_graphs, n, heads) if with_ae else (0,)),
            xs.new_empty((num_graphs, _oc(heads, channels, concat))))


@_impl("gat_wgrad_bf16b")
def _gat_wgrad_bf16b(x_b, dxs_b, W, att_src, att_dst, dbias_partial, heads, channels, gW,
                     g_att_src, g_att_dst, g_bias):
    """gat_wgrad in the bf16 mode on operands already in bf16: x_b from
    project_bf16_export, dxs_b from gat_attn_bwd_bf16dx
    (sv2n_gat_wgrad_node_bf16b)."""
    lib = _lib.load()
    _f32(W, att_src, att_dst, dbias_partial, gW, g_att_src, g_att_dst, g_bias)
    _dense(x_b, dxs_b, W, att_src, att_dst, dbias_partial, gW, g_att_src, g_att_dst, g_bias)
    _need(x_b.dtype == torch.bfloat16 and dxs_b.dtype == torch.bfloat16, "bf16 operands")
    N = x_b.shape[0]
    HC = heads * channels
    F = W.shape[1]
    ldx = (HC + 2 * heads + 3) // 4 * 4
    _need(W.shape[0] == HC and dxs_b.shape[0] == N and dxs_b.shape[1] >= ldx and
          x_b.shape[1] >= F, "W / x_b / dxs_b shapes")
    _need(gW.shape == W.shape, "gW shape")
    ws_n = lib.sv2n_gat_wgrad_node_bf16_workspace(N, F, ldx, heads, channels)
    ws = torch.empty(max(ws_n, 1), device=x_b.device)
    B, OC = dbias_partial.shape
    _lib.check(lib.sv2n_gat_wgrad_node_bf16b(
        x_b.data_ptr(), x_b.stride(0), dxs_b.data_ptr(), dxs_b.stride(0), N, F, ldx,
        W.data_ptr(), att_src.data_ptr(), att_dst.data_ptr(), heads, channels,
        dbias_partial.data_ptr(), B, OC, gW.data_ptr(), _p(g_att_src), _p(g_att_dst),
        _p(g_bias), ws.data_ptr(), ws_n, _st(x_b)), "sv2n_gat_wgrad_node_bf16b")


@_fake("gat_wgrad_bf16b")
def _gat_wgrad_bf16b_fake(x_b, dxs_b, W, att_src, att_dst, dbias_partial, heads, channels, gW,
                          g_att_src, g_att_dst, g_bias):
    return None


def attn_bwd_edge_supported(num_graphs: int, n: int, heads: int, channels: int, edge_dim: int,
                            hl_pad: int) -> bool:
    """Whether sv2n_gat_attn_bwd_edge runs this shape (include/sv2n.h)."""
    return bool(_lib.load().sv2n_gat_attn_bwd_edge_supported(num_graphs, n, heads, channels,
                                                             edge_dim, hl_pad))


@_impl("gat_attn_bwd_edge")
def _gat_attn_bwd_edge(dy, y, xs, psave, keep, keep_scale, edge_attr, dae, layer, hl_pad,
                       num_graphs, n, heads, channels, concat, act, slope, post_u=None,
                       post_p=0.0):
    """gat_attn_bwd of canonical complete graphs with the edge-logit weight
    gradient of every layer fused in (sv2n_gat_attn_bwd_edge, then the
    graph-order sum sv2n_edge_partials_reduce): returns dxs, the bias partials
    and the [edge_dim][hl_pad] gradient edge_logits_bwd would return."""
    lib = _lib.load()
    _f32(dy, y, xs, psave, post_u, edge_attr)
    N, OC = num_graphs * n, _oc(heads, channels, concat)
    E0 = n * (n - 1)
    _rows(xs, N, heads * channels + 2 * heads, "xs")
    _dense(dy, y, psave, keep, post_u, edge_attr, *[d for d in dae if d is not None])
    _need(dy.numel() == N * OC and y.numel() == N * OC, "dy / y shape")
    _need(post_u is None or (post_u.numel() == N * OC and 0.0 <= post_p < 1.0), "post_u / post_p")
    _need(psave.numel() == num_graphs * heads * 1024, "psave shape")
    _need(keep is None or keep.numel() == num_graphs * heads * 1024, "keep shape")
    _need(edge_attr.dim() == 2 and edge_attr.shape[0] == num_graphs * E0, "edge_attr rows")
    L = len(dae)
    _need(0 <= layer < L and all((d is None) == (k == layer) for k, d in enumerate(dae)),
          "dae: one tensor per other layer, None for this one")
    _need(all(d.numel() == num_graphs * E0 * heads for d in dae if d is not None), "dae shape")
    D = edge_attr.shape[1]
    dev = xs.device
    dxs = torch.empty_like(xs)
    dbp = torch.empty(num_graphs, OC, device=dev)
    part = torch.empty(num_graphs, D * hl_pad, device=dev)
    dwf = torch.empty(D, hl_pad, device=dev)
    ptrs = _lib.ptr_array([0 if d is None else d.data_ptr() for d in dae])
    st = _st(xs)
    _lib.check(lib.sv2n_gat_attn_bwd_edge(
        dy.data_ptr(), y.data_ptr(), xs.data_ptr(), xs.stride(0), psave.data_ptr(), _p(keep),
        keep_scale, _p(post_u), post_p, dxs.data_ptr(), dbp.data_ptr(), edge_attr.data_ptr(), D,
        ptrs, L, layer, hl_pad, part.data_ptr(), num_graphs, n, heads, channels, int(concat), act,
        slope, st), "sv2n_gat_attn_bwd_edge")
    _lib.check(lib.sv2n_edge_partials_reduce(part.data_ptr(), num_graphs, D * hl_pad,
                                             dwf.data_ptr(), st), "sv2n_edge_partials_reduce")
    return dxs, dbp, dwf


@_fake("gat_attn_bwd_edge")
def _gat_attn_bwd_edge_fake(dy, y, xs, psave, keep, keep_scale, edge_attr, dae, layer, hl_pad,
                            num_graphs, n, heads, channels, concat, act, slope, post_u=None,
                            post_p=0.0):
    return (torch.empty_like(xs), xs.new_empty((num_graphs, _oc(heads, channels, concat))),
            xs.new_empty((edge_attr.shape[1], hl_pad)))


@_impl("gat_attn_tiled_bwd")
def _gat_attn_tiled_bwd(dy, y, xs, ae, num_edges, eid, keep, keep_scale, rowmask, num_graphs, n,
                        heads, channels, concat, act, slope):
    lib = _lib.load()
    _f32(dy, y, xs, ae)
    N, OC = num_graphs * n, _oc(heads, channels, concat)
    _rows(xs, N, heads * channels + 2 * heads, "xs")
    _dense(dy, y, ae, eid, keep, rowmask)
    _need(dy.numel() == N * OC and y.numel() == N * OC, "dy / y shape")
    _need(ae is None or ae.numel() == heads * num_edges, "ae shape")
    _need(eid is None or eid.numel() == N * n, "eid shape")
    dev = xs.device
    dxs = torch.empty_like(xs)
    dae = torch.empty(heads, num_edges, device=dev) if (ae is not None and num_edges > 0) else \
        torch.empty(0, device=dev)
    dbp = torch.empty(num_graphs, _oc(heads, channels, concat), device=dev)
    _lib.check(lib.sv2n_gat_attn_tiled_bwd(
        dy.data_ptr(), y.data_ptr(), xs.data_ptr(), xs.stride(0), _p(ae), num_edges, _p(eid),
        _p(keep), keep_scale, _p(rowmask), dxs.data_ptr(), _p(dae), dbp.data_ptr(), num_graphs,
        n, heads, channels, int(concat), act, slope, _st(xs)), "sv2n_gat_attn_tiled_bwd")
    return dxs, dae, dbp


@_fake("gat_attn_tiled_bwd")
def _gat_attn_tiled_bwd_fake(dy, y, xs, ae, num_edges, eid, keep, keep_scale, rowmask,
                             num_graphs, n, heads, channels, concat, act, slope):
    return (torch.empty_like(xs),
            xs.new_empty((heads, num_edges) if (ae is not None and num_edges > 0) else (0,)),
            xs.new_empty((num_graphs, _oc(heads, channels, concat))))


# --------------------------------------------------------------------------
# weight gradients of one layer (sv2n_gat_wgrad_node / _bf16), accumulating
# --------------------------------------------------------------------------
@_impl("gat_wgrad")
def _gat_wgrad(x, dxs, W, att_src, att_dst, dbias_partial, heads, channels, bf16, gW, g_att_src,
               g_att_dst, g_bias):
    lib = _lib.load()
    _f32(x, dxs, W, att_src, att_dst, dbias_partial, gW, g_att_src, g_att_dst, g_bias)
    _dense(dxs, W, att_src, att_dst, dbias_partial, gW, g_att_src, g_att_dst, g_bias)
    N, ldx = dxs.shape
    F = W.shape[1]
    HC = heads * channels
    _need(W.shape[0] == HC and ldx >= HC + 2 * heads, "W / dxs shapes")
    if x is not None:
        _rows(x, N, F, "x")
    _need(gW is None or gW.shape == W.shape, "gW shape")
    _need(g_att_src is None or g_att_src.numel() == HC, "g_att_src shape")
    _need(g_att_dst is None or g_att_dst.numel() == HC, "g_att_dst shape")
    weights = gW is not None or g_att_src is not None or g_att_dst is not None
    _need(x is not None or not weights, "x is required for weight gradients")
    use_bf16 = bf16 and weights and x.stride(0) % 4 == 0 and F >= 4 and \
        x.data_ptr() % 16 == 0 and dxs.data_ptr() % 16 == 0
    ws_fn = lib.sv2n_gat_wgrad_node_bf16_workspace if use_bf16 else \
        lib.sv2n_gat_wgrad_node_workspace
    fn = lib.sv2n_gat_wgrad_node_bf16 if use_bf16 else lib.sv2n_gat_wgrad_node
    ws_n = ws_fn(N, F, ldx, heads, channels)
    ws = torch.empty(max(ws_n, 1), device=dxs.device)
    B, OC = dbias_partial.shape
    _lib.check(fn(_p(x) if weights else None, x.stride(0) if weights else 0, dxs.data_ptr(), ldx,
                  N, F, W.data_ptr(), att_src.data_ptr(), att_dst.data_ptr(), heads, channels,
                  dbias_partial.data_ptr(), B, OC, _p(gW), _p(g_att_src), _p(g_att_dst),
                  _p(g_bias), ws.data_ptr(), ws_n, _st(dxs)), "sv2n_gat_wgrad_node")


@_fake("gat_wgrad")
def _gat_wgrad_fake(x, dxs, W, att_src, att_dst, dbias_partial, heads, channels, bf16, gW,
                    g_att_src, g_att_dst, g_bias):
    return None


# --------------------------------------------------------------------------
# output head (sv2n_head_*), fused with the MSE loss
# --------------------------------------------------------------------------
@_impl("head_fwd")
def _head_fwd(x, weight, bias):
    lib = _lib.load()
    _f32(x, weight, bias)
    _dense(x, weight, bias)
    N, C = x.shape
    O = weight.shape[0]
    _need(weight.shape[1] == C and (bias is None or bias.numel() == O), "head shapes")
    out = torch.empty(N, O, device=x.device)
    _lib.check(lib.sv2n_head_fwd(x.data_ptr(), N, C, weight.data_ptr(), _p(bias), O,
                                 out.data_ptr(), _st(x)), "sv2n_head_fwd")
    return out


@_fake("head_fwd")
def _head_fwd_fake(x, weight, bias):
    return x.new_empty((x.shape[0], weight.shape[0]))


@_impl("head_bwd")
def _head_bwd(x, weight, dout, g_weight, g_bias):
    lib = _lib.load()
    _dense(x, weight, g_weight, g_bias)
    N, C = x.shape
    O = weight.shape[0]
    dout = dout.contiguous()
    _need(dout.numel() == N * O, "dout shape")
    dx = torch.empty_like(x)
    ws_n = lib.sv2n_head_bwd_workspace(N, C, O)
    ws = _lib.persistent_zeros("head", ws_n, x.device)
    _lib.check(lib.sv2n_head_bwd(x.data_ptr(), N, C, weight.data_ptr(), O, dout.data_ptr(),
                                 dx.data_ptr(), _p(g_weight), _p(g_bias), ws.data_ptr(), ws_n,
                                 _st(x)), "sv2n_head_bwd")
    return dx


@_fake("head_bwd")
def _head_bwd_fake(x, weight, dout, g_weight, g_bias):
    return torch.empty_like(x)


@_impl("head_mse_fwd")
def _head_mse_fwd(x, weight, bias, target, loss_sum=None):
    lib = _lib.load()
    _f32(x, weight, bias, target)
    _dense(x, weight, bias)
    N, C = x.shape
    O = weight.shape[0]
    target = target.reshape(-1).contiguous()
    _need(target.numel() == N * O, f"target has {target.numel()} elements, expected {N * O}")
    diff = torch.empty(N * O, device=x.device)
    loss = torch.empty((), device=x.device)
    ws_n = lib.sv2n_head_mse_workspace(N, C, O)
    ws = _lib.persistent_zeros("head", ws_n, x.device)
    _lib.check(lib.sv2n_head_mse_fwd(x.data_ptr(), N, C, weight.data_ptr(), _p(bias), O,
                                     target.data_ptr(), None, diff.data_ptr(), loss.data_ptr(),
                                     _p(loss_sum), ws.data_ptr(), ws_n, _st(x)),
               "sv2n_head_mse_fwd")
    return loss, diff


@_fake("head_mse_fwd")
def _head_mse_fwd_fake(x, weight, bias, target, loss_sum=None):
    return x.new_empty(()), x.new_empty((x.shape[0] * weight.shape[0],))


@_impl("head_mse_bwd")
def _head_mse_bwd(x, weight, diff, grad_loss, g_weight, g_bias):
    lib = _lib.load()
    _dense(x, weight, diff, g_weight, g_bias)
    N, C = x.shape
    O = weight.shape[0]
    _need(diff.numel() == N * O, "diff shape")
    gl = grad_loss.reshape(()).contiguous().to(torch.float32)
    dx = torch.empty_like(x)
    ws_n = lib.sv2n_head_mse_workspace(N, C, O)
    ws = _lib.persistent_zeros("head", ws_n, x.device)
    _lib.check(lib.sv2n_head_mse_bwd(x.data_ptr(), N, C, weight.data_ptr(), O, diff.data_ptr(),
                                     gl.data_ptr(), dx.data_ptr(), _p(g_weight), _p(g_bias),
                                     ws.data_ptr(), ws_n, _st(x)), "sv2n_head_mse_bwd")
    return dx


@_fake("head_mse_bwd")
def _head_mse_bwd_fake(x, weight, diff, grad_loss, g_weight, g_bias):
    return torch.empty_like(x)


@_impl("head_mse_train")
def _head_mse_train(x, weight, bias, target, g_weight, g_bias, loss_sum=None):
    """Head + MSE forward and backward in one launch (upstream loss gradient
    1): returns (loss, dx) and accumulates the head's parameter gradients."""
    lib = _lib.load()
    _f32(x, weight, bias, target)
    _dense(x, weight, bias, g_weight, g_bias)
    N, C = x.shape
    O = weight.shape[0]
    target = target.reshape(-1).contiguous()
    _need(target.numel() == N * O, f"target has {target.numel()} elements, expected {N * O}")
    loss = torch.empty((), device=x.device)
    dx = torch.empty_like(x)
    ws_n = lib.sv2n_head_mse_train_workspace(N, C, O)
    ws = _lib.persistent_zeros("head", ws_n, x.device)
    _lib.check(lib.sv2n_head_mse_train(x.data_ptr(), N, C, weight.data_ptr(), _p(bias), O,
                                       target.data_ptr(), loss.data_ptr(), _p(loss_sum),
                                       dx.data_ptr(),
                                       _p(g_weight), _p(g_bias), ws.data_ptr(), ws_n, _st(x)),
               "sv2n_head_mse_train")
    return loss, dx


@_fake("head_mse_train")
def _head_mse_train_fake(x, weight, bias, target, g_weight, g_bias, loss_sum=None):
    return x.new_empty(()), torch.empty_like(x)


def head_split_fits(in_features: int, out_features: int) -> bool:
    """Whether sv2n_head_mse_train_rows / _reduce take this head (the
    wave-per-rows kernel: in <= 1024, out <= 4, out * ceil(in / 64) <= 32)."""
    kc = (in_features + 63) // 64
    kc = 1 if kc <= 1 else 2 if kc <= 2 else 4 if kc <= 4 else 8 if kc <= 8 else 16
    return 0 < out_features <= 4 and 0 < in_features <= 1024 and out_features * kc <= 32


def head_split_workspace(num_rows: int, in_features: int, out_features: int,
                         device) -> torch.Tensor:
    """The persistent workspace of the two-launch head (its own key: the
    reduce may still run on a side stream while other head ops run)."""
    n = _lib.load().sv2n_head_mse_train_workspace(num_rows, in_features, out_features)
    return _lib.persistent_zeros("head_split", n, device)


@_impl("head_mse_train_rows")
def _head_mse_train_rows(x, weight, bias, target, ws):
    """First launch of the two-launch head + MSE training step
    (sv2n_head_mse_train_rows): dx, and the block partials in ``ws``."""
    lib = _lib.load()
    _f32(x, weight, bias, target, ws)
    _dense(x, weight, bias, ws)
    N, C = x.shape
    O = weight.shape[0]
    target = target.reshape(-1).contiguous()
    _need(target.numel() == N * O, f"target has {target.numel()} elements, expected {N * O}")
    dx = torch.empty_like(x)
    _lib.check(lib.sv2n_head_mse_train_rows(x.data_ptr(), N, C, weight.data_ptr(), _p(bias), O,
                                            target.data_ptr(), dx.data_ptr(), ws.data_ptr(),
                                            ws.numel(), _st(x)), "sv2n_head_mse_train_rows")
    return dx


@_fake("head_mse_train_rows")
def _head_mse_train_rows_fake(x, weight, bias, target, ws):
    return torch.empty_like(x)


@_impl("head_mse_train_reduce")
def _head_mse_train_reduce(ws, num_rows, in_features, out_features, loss, g_weight, g_bias,
                           loss_sum=None):
    """Second launch (sv2n_head_mse_train_reduce), on the current stream:
    loss, loss_sum and the head's parameter gradients from ``ws``."""
    lib = _lib.load()
    _f32(ws, loss, g_weight, g_bias, loss_sum)
    _dense(ws, loss, g_weight, g_bias, loss_sum)
    need = lib.sv2n_head_mse_train_workspace(num_rows, in_features, out_features)
    if ws.numel() < need:
        raise ValueError(f"head_mse_train_reduce: workspace has {ws.numel()} floats, "
                         f"the shape needs {need}")
    _lib.check(lib.sv2n_head_mse_train_reduce(ws.data_ptr(), ws.numel(), num_rows, in_features,
                                              out_features, loss.data_ptr(), _p(loss_sum),
                                              _p(g_weight), _p(g_bias), _st(ws)),
               "sv2n_head_mse_train_reduce")


@_fake("head_mse_train_reduce")
def _head_mse_train_reduce_fake(ws, num_rows, in_features, out_features, loss, g_weight, g_bias,
                                loss_sum=None):
    return None


# --------------------------------------------------------------------------
# optimizer step and window builder
# --------------------------------------------------------------------------
@_impl("adam_step")
def _adam_step(param, grad, exp_avg, exp_avg_sq, step, ticket, lr, beta1, beta2, eps,
               weight_decay):
    lib = _lib.load()
    _f32(param, grad, exp_avg, exp_avg_sq)
    _dense(param, grad, exp_avg, exp_avg_sq, step, ticket)
    _need(grad.numel() == param.numel() == exp_avg.numel() == exp_avg_sq.numel(), "adam sizes")
    _need(ticket.numel() >= 288 and ticket.dtype == torch.int32, "adam ticket words")
    _lib.check(lib.sv2n_adam_f32_step(param.data_ptr(), grad.data_ptr(), exp_avg.data_ptr(),
                                      exp_avg_sq.data_ptr(), param.numel(), step.data_ptr(),
                                      ticket.data_ptr(), lr, beta1, beta2, eps, weight_decay,
                                      _st(param)), "sv2n_adam_f32_step")


@_impl("dropout_uniform")
def _dropout_uniform(rows, cols, step, seed, salt):
    """[rows][cols] uniforms in [0, 1) from Philox4x32-10 keyed by ``seed``
    with the device step count ``step`` (float32 scalar) and ``salt`` in the
    counter (sv2n_dropout_uniform): a captured step draws fresh values on
    every replay without a torch random op in the graph."""
    lib = _lib.load()
    _need(step.is_cuda and step.dtype == torch.float32 and step.numel() >= 1,
          "step must be a device float32 scalar")
    u = torch.empty(rows, cols, device=step.device)
    _lib.check(lib.sv2n_dropout_uniform(u.data_ptr(), u.numel(), seed & 0xFFFFFFFFFFFFFFFF,
                                        step.data_ptr(), salt & 0xFFFFFFFF, _st(step)),
               "sv2n_dropout_uniform")
    return u


@_fake("dropout_uniform")
def _dropout_uniform_fake(rows, cols, step, seed, salt):
    return step.new_empty(rows, cols)


@_fake("adam_step")
def _adam_step_fake(param, grad, exp_avg, exp_avg_sq, step, ticket, lr, beta1, beta2, eps,
                    weight_decay):
    return None


@_impl("window_gather")
def _window_gather(vol, volvol, starts, seq_length, future_steps, canon, x, edge_attr, y,
                   start_offset=0, diag=None, x_bf16=None, cov_var_only=False, skip_x=False):
    """``cov_var_only``: of edge_attr only what the covariance-layout edge
    passes read (sv2n_window_gather_cv); the caller vouches that nothing
    else reads it (data.WindowDataset.empty_batch(cov_var_only=True)).
    ``skip_x``: only the bf16 twin of x is written (x left as it was; ABI
    21), for a batch whose x is read through the twin alone
    (data.WindowDataset.empty_batch(twin_only=True))."""
    lib = _lib.load()
    _f32(vol, volvol, x, edge_attr, y)
    _need(vol.is_contiguous() and volvol.is_contiguous(), "series must be contiguous")
    _need(starts.dtype == torch.long, "starts must be int64")
    _dense(starts, canon, x, edge_attr, y)
    n, B = vol.shape[1], starts.numel()
    _need(x.numel() == B * n * n * seq_length and
          edge_attr.numel() == B * n * (n - 1) * 3 * seq_length and
          y.numel() == B * n * future_steps, "window output buffer sizes")
    _need(volvol.shape == vol.shape and vol.dim() == 3, "series shapes")
    # windows outside the series come back as NaN (checked in the kernel:
    # the starts live on the device, so no host round trip here)
    if diag is not None:  # the series' diagonal, diag[t][v] = volvol[t][v][v]
        _f32(diag)
        _need(diag.is_contiguous() and diag.shape == vol.shape[:2], "diag must be [T][n]")
    _need(not skip_x or x_bf16 is not None, "skip_x needs x_bf16")
    x_ptr = 0 if skip_x else x.data_ptr()
    if x_bf16 is not None:  # bf16(x) beside x (sv2n_window_gather_bf16x)
        _need(x_bf16.dtype == torch.bfloat16 and x_bf16.dim() == 2 and
              x_bf16.shape[0] == x.shape[0] and x_bf16.stride(1) == 1, "x_bf16 layout")
    if cov_var_only:
        _lib.check(lib.sv2n_window_gather_cv(
            vol.data_ptr(), volvol.data_ptr(), _p(diag), vol.shape[1], vol.shape[0],
            starts.data_ptr(), start_offset, starts.numel(), seq_length, future_steps,
            canon.data_ptr(), x_ptr, _p(x_bf16),
            0 if x_bf16 is None else x_bf16.stride(0), edge_attr.data_ptr(), y.data_ptr(),
            _st(vol)), "sv2n_window_gather_cv")
        return
    if x_bf16 is not None:
        _lib.check(lib.sv2n_window_gather_bf16x(
            vol.data_ptr(), volvol.data_ptr(), _p(diag), vol.shape[1], vol.shape[0],
            starts.data_ptr(), start_offset, starts.numel(), seq_length, future_steps,
            canon.data_ptr(), x_ptr, x_bf16.data_ptr(), x_bf16.stride(0),
            edge_attr.data_ptr(), y.data_ptr(), _st(vol)), "sv2n_window_gather_bf16x")
        return
    _lib.check(lib.sv2n_window_gather_diag(vol.data_ptr(), volvol.data_ptr(), _p(diag),
                                           vol.shape[1], vol.shape[0], starts.data_ptr(),
                                           start_offset, starts.numel(), seq_length,
                                           future_steps, canon.data_ptr(), x.data_ptr(),
                                           edge_attr.data_ptr(), y.data_ptr(), _st(vol)),
               "sv2n_window_gather_diag")


@_fake("window_gather")
def _window_gather_fake(vol, volvol, starts, seq_length, future_steps, canon, x, edge_attr, y,
                        start_offset=0, diag=None, x_bf16=None, cov_var_only=False,
                        skip_x=False):
    return None


def window_bf16x_supported(n: int, seq_length: int, future_steps: int) -> bool:
    """Whether sv2n_window_gather_bf16x takes the shape (include/sv2n.h)."""
    return (n * seq_length) % 4 == 0 and 4 * 3 * seq_length * (n + 1) <= 64 * 1024 \
        and future_steps <= 256


@_impl("project_a16")
def _project_a16(a_bf16, k, planes, w):
    """The bf16-mode projection bf16(a)·wᵀ from a bf16 copy of a ([M][ld],
    the first k columns; sv2n_gemm_bf16_a16)."""
    lib = _lib.load()
    _f32(w)
    _need(a_bf16.dtype == torch.bfloat16 and a_bf16.stride(1) == 1, "a_bf16 layout")
    M = a_bf16.shape[0]
    N = w.shape[0]
    out = torch.empty(M, N, device=a_bf16.device, dtype=torch.float32)
    _lib.check(lib.sv2n_gemm_bf16_a16(a_bf16.data_ptr(), a_bf16.stride(0), planes.data_ptr(),
                                      out.data_ptr(), out.stride(0), M, N, k, _st(a_bf16)),
               "sv2n_gemm_bf16_a16")
    return out


@_fake("project_a16")
def _project_a16_fake(a_bf16, k, planes, w):
    return a_bf16.new_empty((a_bf16.shape[0], w.shape[0]), dtype=torch.float32)


OPS = tuple(_SCHEMAS)
