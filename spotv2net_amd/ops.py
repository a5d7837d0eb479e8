"""Autograd operators over the sv2n C-ABI (include/sv2n.h).

Each ``torch.autograd.Function`` here launches hand-written gfx950 kernels
through ``_lib`` on the current HIP stream; buffers come from PyTorch's caching
allocator, so every op is capturable into a hipGraph.  There is no CPU path:
CPU tensors raise.

Operators
---------
``linear(x, w)``            x @ wᵀ on f32 MFMA (PyG ``Linear``)
``edge_logits(ea, wf, …)``  folded lin_edge·att_edge logits for L layers (a8)
``gat_attention(xs, …)``    self loops + leaky_relu + per-target softmax +
                            dropout + aggregation + concat/mean + bias + act
                            (a7, a9-a11, GATModel act a4)
"""
from __future__ import annotations

import os

from typing import Optional, Sequence

import torch

from . import _lib
from .layout import GraphLayout

ACT_CODES = {None: 0, "identity": 0, "relu": 1, "tanh": 2, "sigmoid": 3}


def _require_device(*ts: Optional[torch.Tensor]) -> torch.device:
    dev = None
    for t in ts:
        if t is None:
            continue
        if t.device.type != "cuda":
            raise RuntimeError(
                "spotv2net_amd runs the GAT hot path only on a ROCm GPU (got a "
                f"{t.device.type} tensor); there is no CPU fallback")
        if t.dtype != torch.float32 and t.is_floating_point():
            raise TypeError(f"spotv2net_amd kernels compute in fp32 (got {t.dtype})")
        dev = t.device
    return dev


def _aligned(t: torch.Tensor) -> torch.Tensor:
    t = t.contiguous()
    if t.data_ptr() % 16:
        t = t.clone()
    return t


def _stream(dev: torch.device) -> int:
    return _lib.stream_handle(dev)


# ---------------------------------------------------------------------------
# GEMM
# ---------------------------------------------------------------------------
def gemm_f32(a: torch.Tensor, a_kmajor: bool, b: torch.Tensor, b_kmajor: bool,
             M: int, N: int, K: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """C[M,N] = Σ_k A(m,k) B(n,k) with A/B given k-major ([rows][K]) or not
    ([K][rows]); thin wrapper of sv2n_gemm_f32."""
    lib = _lib.load()
    dev = a.device
    if out is None:
        out = torch.empty(M, N, device=dev, dtype=torch.float32)
    ws_n = lib.sv2n_gemm_f32_workspace(M, N, K)
    ws = torch.empty(max(ws_n, 1), device=dev, dtype=torch.float32) if ws_n > 0 else None
    _lib.check(lib.sv2n_gemm_f32(int(a_kmajor), int(b_kmajor), a.data_ptr(), a.stride(0),
                                 b.data_ptr(), b.stride(0), out.data_ptr(), out.stride(0),
                                 M, N, K, _lib.ptr(ws), ws_n, _stream(dev)), "sv2n_gemm_f32")
    return out


# Projection GEMMs with a small weight operand run on the bf16-split MFMA
# kernel (sv2n_gemm_f32x3, f32-accurate); SV2N_GEMM=f32 selects the exact-f32
# MFMA kernel instead.
_SPLIT_GEMM = os.environ.get("SV2N_GEMM", "split3").lower() != "f32"


def weight_planes(w: torch.Tensor, transpose: bool) -> torch.Tensor:
    """The three bf16 planes [3][rows][Kp] of a weight used as the B operand of
    sv2n_gemm_f32x3: B(n, k) = w[n][k] (transpose False) or w[k][n] (True)."""
    lib = _lib.load()
    rows, K = (w.shape[1], w.shape[0]) if transpose else (w.shape[0], w.shape[1])
    Kp = lib.sv2n_split3_kpad(K)
    out = torch.empty(3, rows, Kp, device=w.device, dtype=torch.int16)
    _lib.check(lib.sv2n_split3(w.data_ptr(), rows, K, w.stride(0), int(transpose), out.data_ptr(),
                               _stream(w.device)), "sv2n_split3")
    return out


def _split_ok(a: torch.Tensor) -> bool:
    return _SPLIT_GEMM and a.stride(1) == 1 and a.stride(0) % 4 == 0 and a.data_ptr() % 16 == 0


def project(a: torch.Tensor, w: torch.Tensor, transpose_w: bool) -> torch.Tensor:
    """C = a · B with B(n,k) = w[n][k] (C = a·wᵀ) or w[k][n] (C = a·w); a is
    [M][K] k-contiguous.  bf16-split MFMA when a is aligned, else exact f32."""
    M, K = a.shape
    N = w.shape[1] if transpose_w else w.shape[0]
    if _split_ok(a):
        lib = _lib.load()
        planes = weight_planes(w, transpose_w)
        out = torch.empty(M, N, device=a.device, dtype=torch.float32)
        _lib.check(lib.sv2n_gemm_f32x3(a.data_ptr(), a.stride(0), planes.data_ptr(),
                                       out.data_ptr(), out.stride(0), M, N, K,
                                       _stream(a.device)), "sv2n_gemm_f32x3")
        return out
    return gemm_f32(a, True, w, not transpose_w, M, N, K)


def project_planes(a: torch.Tensor, planes: Optional[torch.Tensor], w: torch.Tensor,
                   transpose_w: bool) -> torch.Tensor:
    """project(a, w, transpose_w) with w's bf16 split planes already made
    (sv2n_gat_prep_fwd_all); exact-f32 fallback on w as in project()."""
    if planes is None or not _split_ok(a):
        return project(a, w, transpose_w)
    lib = _lib.load()
    M, K = a.shape
    N = w.shape[1] if transpose_w else w.shape[0]
    out = torch.empty(M, N, device=a.device, dtype=torch.float32)
    _lib.check(lib.sv2n_gemm_f32x3(a.data_ptr(), a.stride(0), planes.data_ptr(), out.data_ptr(),
                                   out.stride(0), M, N, K, _stream(a.device)), "sv2n_gemm_f32x3")
    return out


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
        x = x.contiguous()
        w = w.contiguous()
        M, K = x.shape
        N = w.shape[0]
        y = gemm_f32(x, True, w, True, M, N, K)
        ctx.save_for_backward(x, w)
        return y

    @staticmethod
    def backward(ctx, dy: torch.Tensor):
        x, w = ctx.saved_tensors
        dy = dy.contiguous()
        M, K = x.shape
        N = w.shape[0]
        dx = dw = None
        if ctx.needs_input_grad[0]:
            # dx[m,k] = Σ_o dy[m,o] w[o,k]
            dx = gemm_f32(dy, True, w, False, M, K, N)
        if ctx.needs_input_grad[1]:
            # dwᵀ[k,o] = Σ_m x[m,k] dy[m,o]
            dwt = gemm_f32(x, False, dy, False, K, N, M)
            dw = dwt.t()
        return dx, dw


def linear(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    _require_device(x, w)
    return _Linear.apply(x, w)


# ---------------------------------------------------------------------------
# edge logits
# ---------------------------------------------------------------------------
def pad_columns(w: torch.Tensor) -> tuple[torch.Tensor, int]:
    """[D, HL] -> [D, hl_pad] with hl_pad ∈ {4, 8, 16, 32} (zero columns)."""
    hl = w.shape[1]
    for hp in (4, 8, 16, 32):
        if hl <= hp:
            break
    else:
        raise ValueError(f"at most 32 (layers x heads) edge-logit columns supported, got {hl}")
    if hp != hl:
        w = torch.nn.functional.pad(w, (0, hp - hl))
    return w.contiguous(), hp


class _EdgeLogits(torch.autograd.Function):
    @staticmethod
    def forward(ctx, edge_attr: torch.Tensor, wfold: torch.Tensor, layout: GraphLayout,
                num_layers: int, heads: int):
        lib = _lib.load()
        dev = edge_attr.device
        ea = _aligned(edge_attr)
        E, D = ea.shape
        wf, hp = pad_columns(wfold)
        B, n = layout.num_graphs, layout.n
        outs = [torch.empty(B, n, n, heads, device=dev, dtype=torch.float32)
                for _ in range(num_layers)]
        ctx.save_for_backward(ea)
        ctx.layout = layout
        ctx.meta = (num_layers, heads, hp, wfold.shape[1])
        if E == 0:  # no edges: the attention kernels never read ae
            return tuple(outs)
        ptrs = _lib.ptr_array([o.data_ptr() for o in outs])
        ei = layout.edge_index if layout.kind == "block" else None
        _lib.check(lib.sv2n_edge_logits_fwd(ea.data_ptr(), E, D, _lib.ptr(ei),
                                            layout.canon.data_ptr(), wf.data_ptr(), hp, ptrs,
                                            num_layers, heads, B, n, _stream(dev)),
                   "sv2n_edge_logits_fwd")
        return tuple(outs)

    @staticmethod
    def backward(ctx, *grads):
        (ea,) = ctx.saved_tensors
        layout: GraphLayout = ctx.layout
        L, H, hp, hl = ctx.meta
        lib = _lib.load()
        dev = ea.device
        E, D = ea.shape
        B, n = layout.num_graphs, layout.n
        if E == 0:
            return None, torch.zeros(D, hl, device=dev, dtype=torch.float32), None, None, None
        gs = [g.contiguous() if g is not None else
              torch.zeros(B, n, n, H, device=dev, dtype=torch.float32) for g in grads]
        ptrs = _lib.ptr_array([g.data_ptr() for g in gs])
        ws_n = lib.sv2n_edge_logits_bwd_workspace(D, hp)
        ws = torch.empty(ws_n, device=dev, dtype=torch.float32)
        dwf = torch.empty(D, hp, device=dev, dtype=torch.float32)
        ei = layout.edge_index if layout.kind == "block" else None
        _lib.check(lib.sv2n_edge_logits_bwd(ea.data_ptr(), E, D, _lib.ptr(ei),
                                            layout.canon.data_ptr(), ptrs, L, H, B, n,
                                            ws.data_ptr(), ws_n, dwf.data_ptr(), hp,
                                            _stream(dev)), "sv2n_edge_logits_bwd")
        return None, dwf[:, :hl], None, None, None


def edge_logits(edge_attr: torch.Tensor, wfold: torch.Tensor, layout: GraphLayout,
                num_layers: int, heads: int) -> Sequence[torch.Tensor]:
    """Per-layer dense edge logits [B, n, n, H] for the L layers whose folded
    edge weights are the column blocks of ``wfold`` [D, L*H]."""
    _require_device(edge_attr, wfold)
    if edge_attr.requires_grad:
        raise NotImplementedError("gradients w.r.t. edge_attr are not supported (the reference "
                                  "treats edge_attr as data)")
    if edge_attr.dim() == 1:
        edge_attr = edge_attr.view(-1, 1)
    if edge_attr.size(0) != layout.num_edges:
        raise ValueError("edge_attr rows must match edge_index columns")
    return _EdgeLogits.apply(edge_attr, wfold, layout, num_layers, heads)


# ---------------------------------------------------------------------------
# fused attention
# ---------------------------------------------------------------------------
class _GatAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, xs, ae, bias, layout: GraphLayout, heads: int, channels: int, concat: bool,
                act: int, slope: float, keep: Optional[torch.Tensor], keep_scale: float):
        lib = _lib.load()
        dev = xs.device
        B, n = layout.num_graphs, layout.n
        N = layout.num_nodes
        OC = heads * channels if concat else channels
        y = torch.empty(N, OC, device=dev, dtype=torch.float32)
        psave = torch.empty(B, heads, 32, 32, device=dev, dtype=torch.float32)
        ae_c = ae.contiguous() if ae is not None else None
        _lib.check(lib.sv2n_gat_attn_fwd(xs.data_ptr(), xs.stride(0), _lib.ptr(ae_c),
                                         _lib.ptr(layout.rowmask), _lib.ptr(bias), _lib.ptr(keep),
                                         keep_scale, y.data_ptr(), psave.data_ptr(), B, n, heads,
                                         channels, int(concat), act, slope, _stream(dev)),
                   "sv2n_gat_attn_fwd")
        ctx.save_for_backward(xs, y, psave, keep)
        ctx.layout = layout
        ctx.meta = (heads, channels, concat, act, slope, keep_scale, ae is not None,
                    bias is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        xs, y, psave, keep = ctx.saved_tensors
        layout: GraphLayout = ctx.layout
        heads, channels, concat, act, slope, keep_scale, has_ae, has_bias = ctx.meta
        lib = _lib.load()
        dev = xs.device
        B, n = layout.num_graphs, layout.n
        OC = heads * channels if concat else channels
        dy = dy.contiguous()
        dxs = torch.empty_like(xs)
        dae = torch.empty(B, n, n, heads, device=dev, dtype=torch.float32) if has_ae else None
        dbp = torch.empty(B, OC, device=dev, dtype=torch.float32)
        _lib.check(lib.sv2n_gat_attn_bwd(dy.data_ptr(), y.data_ptr(), xs.data_ptr(),
                                         xs.stride(0), psave.data_ptr(), _lib.ptr(keep),
                                         keep_scale, _lib.ptr(layout.rowmask), dxs.data_ptr(),
                                         _lib.ptr(dae), dbp.data_ptr(), B, n, heads, channels,
                                         int(concat), act, slope, _stream(dev)),
                   "sv2n_gat_attn_bwd")
        dbias = dbp.sum(0) if has_bias else None
        return dxs, dae, dbias, None, None, None, None, None, None, None, None


def gat_attention(xs: torch.Tensor, ae: Optional[torch.Tensor], bias: Optional[torch.Tensor],
                  layout: GraphLayout, heads: int, channels: int, concat: bool, act: int,
                  negative_slope: float, attn_dropout: float = 0.0,
                  training: bool = False) -> torch.Tensor:
    """Fused GAT attention for one layer; ``xs`` = [lin_src(x) | a_src | a_dst]."""
    _require_device(xs, ae, bias)
    if layout.tiled:
        from .layout import UnsupportedLayout
        raise UnsupportedLayout("the per-op attention covers n <= 32; larger blocks run through "
                                "the fused stack (GATConv.forward / gat_stack)")
    if xs.stride(1) != 1 or xs.stride(0) % 4 or xs.data_ptr() % 16:
        xs = _aligned(xs)
    keep, scale = None, 1.0
    if training and attn_dropout > 0.0:
        B, n = layout.num_graphs, layout.n
        if attn_dropout >= 1.0:
            keep = torch.zeros(B, heads, 32, 32, device=xs.device, dtype=torch.uint8)
            scale = 0.0
        else:
            keep = (torch.rand(B, heads, 32, 32, device=xs.device) >= attn_dropout).to(torch.uint8)
            scale = 1.0 / (1.0 - attn_dropout)
    return _GatAttention.apply(xs, ae, bias, layout, heads, channels, bool(concat), int(act),
                               float(negative_slope), keep, float(scale))
