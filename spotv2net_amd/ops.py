"""Autograd operators over the sv2n C-ABI (include/sv2n.h).

Each ``torch.autograd.Function`` here launches hand-written gfx950 kernels
through ``_lib`` on the current HIP stream; buffers come from PyTorch's caching
allocator, so every op is capturable into a hipGraph.  There is no CPU path:
CPU tensors raise.

Operators
---------
``linear(x, w)``              x @ wᵀ on f32 MFMA (PyG ``Linear``)
``project / project_planes``  the projection GEMMs of the fused stack
``pad_columns``               edge-fold column padding (a8)

The GAT layers themselves (a7-a12) run as one fused node: ``stack.gat_stack``.
"""
from __future__ import annotations

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
# kernel (sv2n_gemm_f32x3, f32-accurate) whenever the activation operand is
# 16-B aligned with a row stride of whole 16-B chunks; the exact-f32 MFMA
# kernel (sv2n_gemm_f32) takes the rest.


def weight_planes(w: torch.Tensor, transpose: bool) -> torch.Tensor:
    """The three bf16 planes [3][rows][Kp] of a weight used as the B operand of
    sv2n_gemm_f32x3: B(n, k) = w[n][k] (transpose False) or w[k][n] (True)."""
    lib = _lib.load()
    _has_data(w)
    rows, K = (w.shape[1], w.shape[0]) if transpose else (w.shape[0], w.shape[1])
    Kp = lib.sv2n_split3_kpad(K)
    out = torch.empty(3, rows, Kp, device=w.device, dtype=torch.int16)
    _lib.check(lib.sv2n_split3(w.data_ptr(), rows, K, w.stride(0), int(transpose), out.data_ptr(),
                               _stream(w.device)), "sv2n_split3")
    return out


def _has_data(w: torch.Tensor) -> None:
    if w.dim() == 2 and w.numel() > 1 and w.stride() == (0, 0):
        raise RuntimeError("sv2n: Waug placeholder of bf16-mode gat_prep has no data; "
                           "pass the layer's planes")


def _split_ok(a: torch.Tensor) -> bool:
    return a.stride(1) == 1 and a.stride(0) % 4 == 0 and a.data_ptr() % 16 == 0


def project(a: torch.Tensor, w: torch.Tensor, transpose_w: bool) -> torch.Tensor:
    """C = a · B with B(n,k) = w[n][k] (C = a·wᵀ) or w[k][n] (C = a·w); a is
    [M][K] k-contiguous.  bf16-split MFMA when a is aligned, else exact f32."""
    M, K = a.shape
    N = w.shape[1] if transpose_w else w.shape[0]
    _has_data(w)
    if _split_ok(a):
        lib = _lib.load()
        planes = weight_planes(w, transpose_w)
        out = torch.empty(M, N, device=a.device, dtype=torch.float32)
        _lib.check(lib.sv2n_gemm_f32x3(a.data_ptr(), a.stride(0), planes.data_ptr(),
                                       out.data_ptr(), out.stride(0), M, N, K,
                                       _stream(a.device)), "sv2n_gemm_f32x3")
        return out
    return gemm_f32(a, True, w, not transpose_w, M, N, K)


def relu_mask_fusable(a: torch.Tensor, planes: Optional[torch.Tensor], bf16: bool) -> bool:
    """Whether project_planes(..., relu_y) runs the masked f32 GEMM
    (sv2n_gemm_f32x3_relu: the split planes exist, A is 16-B rows, K % 4 == 0)."""
    return not bf16 and planes is not None and _split_ok(a) and a.shape[1] % 4 == 0


def project_planes(a: torch.Tensor, planes: Optional[torch.Tensor], w: torch.Tensor,
                   transpose_w: bool, bf16: bool = False,
                   relu_y: Optional[torch.Tensor] = None) -> torch.Tensor:
    """project(a, w, transpose_w) with w's bf16 split planes already made
    (sv2n_gat_prep_fwd_all); exact-f32 fallback on w as in project().
    ``bf16``: the bf16 execution mode (sv2n_gemm_bf16: bf16 operands, fp32
    accumulation, on plane 0 = bf16_rn(w)).  ``relu_y`` [M][N]: the result
    is masked by relu_y > 0 (ReLU's backward, in the GEMM's store when
    relu_mask_fusable, else as a separate elementwise step)."""
    lib = _lib.load()
    M, K = a.shape
    N = w.shape[1] if transpose_w else w.shape[0]
    if relu_y is not None:
        if relu_y.shape != (M, N) or relu_y.stride(1) != 1:
            raise ValueError(f"relu_y: expected [{M}, {N}] rows, got {tuple(relu_y.shape)}")
        if relu_mask_fusable(a, planes, bf16):
            out = torch.empty(M, N, device=a.device, dtype=torch.float32)
            _lib.check(lib.sv2n_gemm_f32x3_relu(a.data_ptr(), a.stride(0), planes.data_ptr(),
                                                out.data_ptr(), out.stride(0), M, N, K,
                                                relu_y.data_ptr(), relu_y.stride(0),
                                                _stream(a.device)), "sv2n_gemm_f32x3_relu")
            return out
        out = project_planes(a, planes, w, transpose_w, bf16)
        return torch.where(relu_y > 0, out, torch.zeros_like(out))
    if bf16:
        if planes is None:
            planes = weight_planes(w, transpose_w)
        if not (a.stride(1) == 1 and a.stride(0) % 4 == 0 and a.data_ptr() % 16 == 0):
            a = _aligned(a) if a.size(1) % 4 == 0 else \
                torch.nn.functional.pad(a, (0, (-a.size(1)) % 4))[:, :K]
        out = torch.empty(M, N, device=a.device, dtype=torch.float32)
        _lib.check(lib.sv2n_gemm_bf16(a.data_ptr(), a.stride(0), planes.data_ptr(),
                                      out.data_ptr(), out.stride(0), M, N, K, _stream(a.device)),
                   "sv2n_gemm_bf16")
        return out
    if planes is None or not _split_ok(a):
        return project(a, w, transpose_w)
    out = torch.empty(M, N, device=a.device, dtype=torch.float32)
    _lib.check(lib.sv2n_gemm_f32x3(a.data_ptr(), a.stride(0), planes.data_ptr(), out.data_ptr(),
                                   out.stride(0), M, N, K, _stream(a.device)), "sv2n_gemm_f32x3")
    return out


PRECISIONS = ("f32", "bf16")


def resolve_precision(precision: Optional[str]) -> str:
    """The execution mode of a fused GAT node: an explicit ``precision``, else
    bf16 inside ``torch.autocast("cuda", dtype=torch.bfloat16)`` (the
    reference run with autocast, BASELINE config C3), else f32."""
    if precision is not None:
        if precision not in PRECISIONS:
            raise ValueError(f"precision must be one of {PRECISIONS}, got {precision!r}")
        return precision
    if torch.is_autocast_enabled("cuda") and \
            torch.get_autocast_dtype("cuda") == torch.bfloat16:
        return "bf16"
    return "f32"


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
