"""ctypes binding of the C-ABI in ``include/sv2n.h`` (``libsv2n.so``).

This is the one place the Python host side touches native code.  The library
is built in-tree (``make`` / ``__graft_entry__.build()``) for gfx950; if it is
missing or stale the import fails loudly — there is no CPU or eager-PyTorch
fallback for the hot path.
"""
from __future__ import annotations

import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# SV2N_LIB: an alternative build of the same library (diagnostic builds, e.g.
# tools/stamps.py); default the in-tree one
LIB_PATH = os.environ.get("SV2N_LIB") or os.path.join(_HERE, "libsv2n.so")
ABI_VERSION = 21

_c_f = ctypes.POINTER(ctypes.c_float)
_p = ctypes.c_void_p
_i64 = ctypes.c_int64
_i32 = ctypes.c_int
_f32 = ctypes.c_float
_u32 = ctypes.c_uint32
_u64 = ctypes.c_uint64

class PrepLayer(ctypes.Structure):
    """sv2n_prep_layer (include/sv2n.h)."""
    _fields_ = [
        ("W", _p), ("att_src", _p), ("att_dst", _p),
        ("heads", _i32), ("channels", _i32), ("in_features", _i32), ("ldx", _i32),
        ("waug", _p), ("planes", _p), ("planes_t", _p),
        ("W_edge", _p), ("att_edge", _p),
        ("edge_dim", _i32), ("hl_pad", _i32), ("col0", _i32),
        ("wfold", _p), ("nplanes", _i32),
    ]


class EdgeGradLayer(ctypes.Structure):
    """sv2n_edge_grad_layer (include/sv2n.h)."""
    _fields_ = [
        ("W_edge", _p), ("att_edge", _p), ("gW_edge", _p), ("g_att_edge", _p),
        ("heads", _i32), ("channels", _i32), ("col0", _i32),
    ]


# name -> (restype, argtypes); mirrors include/sv2n.h
_SIGNATURES = {
    "sv2n_abi_version": (_i32, []),
    "sv2n_strerror": (ctypes.c_char_p, [_i32]),
    "sv2n_edge_logits_fwd": (_i32, [_p, _i64, _i32, _p, _p, _p, _i32, _p, _i32, _i32, _i64, _i32, _p]),
    "sv2n_edge_logits_bwd_workspace": (_i64, [_i32, _i32]),
    "sv2n_edge_logits_bwd": (_i32, [_p, _i64, _i32, _p, _p, _p, _i32, _i32, _i64, _i32, _p, _i64, _p,
                                    _i32, _p]),
    "sv2n_gat_attn_fwd": (_i32, [_p, _i32, _p, _i32, _p, _p, _p, _f32, _p, _p, _p, _f32, _p, _i64,
                                 _i32, _i32, _i32, _i32, _i32, _f32, _p]),
    "sv2n_gat_attn_bwd": (_i32, [_p, _p, _p, _i32, _p, _p, _f32, _p, _f32, _p, _p, _p, _i32, _p,
                                 _i64, _i32, _i32, _i32, _i32, _i32, _f32, _p]),
    # dy y xs ldx psave keep keep_scale post_u post_p rowmask dxb ld dae eo dbp B n H C concat
    # act slope stream
    "sv2n_gat_attn_bwd_bf16dx": (_i32, [_p, _p, _p, _i32, _p, _p, _f32, _p, _f32, _p, _p, _i32,
                                        _p, _i32, _p, _i64, _i32, _i32, _i32, _i32, _i32, _f32,
                                        _p]),
    "sv2n_gat_attn_fwd_head_mse_supported": (_i32, [_i64, _i32, _i32, _i32, _i32]),
    "sv2n_gat_attn_fwd_head_mse_workspace": (_i64, [_i64, _i32, _i32, _i32]),
    # xs ldx ae eo rowmask bias keep keep_scale dz psave post_u post_p hw hb target loss
    # ghw ghb ws ws_n B n H C concat act slope stream
    "sv2n_gat_attn_fwd_head_mse": (_i32, [_p, _i32, _p, _i32, _p, _p, _p, _f32, _p, _p, _p, _f32,
                                          _p, _p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i32,
                                          _i32, _i32, _i32, _i32, _f32, _p]),
    "sv2n_gat_attn_bwd_edge_supported": (_i32, [_i64, _i32, _i32, _i32, _i32, _i32]),
    # dy y xs ldx psave keep keep_scale post_u post_p dxs dbp ea D layer_dae L layer hlp part
    # B n H C concat act slope stream
    "sv2n_gat_attn_bwd_edge": (_i32, [_p, _p, _p, _i32, _p, _p, _f32, _p, _f32, _p, _p, _p, _i32,
                                      _p, _i32, _i32, _i32, _p, _i64, _i32, _i32, _i32, _i32,
                                      _i32, _f32, _p]),
    "sv2n_edge_partials_reduce": (_i32, [_p, _i64, _i64, _p, _p]),
    "sv2n_gat_attn_tiled_workspace": (_i64, [_i64, _i32, _i32, _i32, _i32]),
    "sv2n_gat_attn_tiled_fwd": (_i32, [_p, _i32, _p, _i64, _p, _p, _p, _p, _f32, _p, _p, _i64,
                                       _i64, _i32, _i32, _i32, _i32, _i32, _f32, _p]),
    "sv2n_gat_attn_tiled_bwd": (_i32, [_p, _p, _p, _i32, _p, _i64, _p, _p, _f32, _p, _p, _p, _p,
                                       _i64, _i32, _i32, _i32, _i32, _i32, _f32, _p]),
    "sv2n_gat_attn_fused_supported": (_i32, [_i32, _i32, _i32, _i32]),
    "sv2n_gat_attn_fused_fwd": (_i32, [_p, _i32, _p, _i32, _p, _i32, _i32, _p, _p, _p, _f32, _p, _p,
                                       _p, _i64, _i32, _i32, _i32, _i32, _i32, _f32, _p]),
    "sv2n_gat_attn_fused_bwd_workspace": (_i64, [_i64, _i32, _i32, _i32, _i32]),
    "sv2n_gat_attn_fused_bwd": (_i32, [_p, _p, _p, _p, _p, _i32, _p, _i32, _p, _i32, _i32, _p, _p,
                                       _f32, _p, _p, _p, _p, _i64, _i64, _i32, _i32, _i32, _i32,
                                       _i32, _f32, _p]),
    "sv2n_edge_logits_fwd_planes": (_i32, [_p, _i64, _i32, _p, _i32, _p, _i32, _i32, _p]),
    "sv2n_edge_logits_bwd_planes": (_i32, [_p, _i64, _i32, _p, _p, _i32, _i32, _p, _i64, _p,
                                           _i32, _p]),
    "sv2n_block_eid": (_i32, [_p, _i64, _i64, _i32, _p, _p]),
    "sv2n_split3_kpad": (_i64, [_i64]),
    "sv2n_split3": (_i32, [_p, _i64, _i64, _i64, _i32, _p, _p]),
    "sv2n_gemm_f32x3": (_i32, [_p, _i64, _p, _p, _i64, _i64, _i64, _i64, _p]),
    "sv2n_gemm_f32x3_relu": (_i32, [_p, _i64, _p, _p, _i64, _i64, _i64, _i64, _p, _i64, _p]),
    "sv2n_gemm_bf16": (_i32, [_p, _i64, _p, _p, _i64, _i64, _i64, _i64, _p]),
    "sv2n_gemm_bf16_export": (_i32, [_p, _i64, _p, _p, _i64, _i64, _i64, _i64, _p, _i64, _p]),
    "sv2n_gemm_bf16_a16": (_i32, [_p, _i64, _p, _p, _i64, _i64, _i64, _i64, _p]),
    "sv2n_gemm_f32_workspace": (_i64, [_i64, _i64, _i64]),
    "sv2n_gemm_f32_slabs_count": (_i32, [_i64, _i64, _i64]),
    "sv2n_gemm_f32_slabs": (_i32, [_i32, _i32, _p, _i64, _p, _i64, _i64, _i64, _i64, _p, _i64, _p]),
    "sv2n_gemm_f32": (_i32, [_i32, _i32, _p, _i64, _p, _i64, _p, _i64, _i64, _i64, _i64, _p, _i64, _p]),
    "sv2n_block_rowmask": (_i32, [_p, _i64, _i64, _i32, _p, _p]),
    "sv2n_block_rowmask_checked": (_i32, [_p, _i64, _i64, _i32, _p, _p, _p]),
    "sv2n_gat_prep_fwd": (_i32, [_p, _p, _p, _i32, _i32, _i32, _p, _i32, _p, _p, _i32, _p, _i32,
                                 _i32, _p]),
    "sv2n_gat_prep_bwd_workspace": (_i64, [_i32, _i32]),
    "sv2n_gat_prep_fwd_all": (_i32, [_p, _i32, _p]),
    "sv2n_gat_wgrad_node_workspace": (_i64, [_i64, _i32, _i32, _i32, _i32]),
    "sv2n_gat_wgrad_node": (_i32, [_p, _i64, _p, _i32, _i64, _i32, _p, _p, _p, _i32, _i32, _p,
                                   _i32, _i32, _p, _p, _p, _p, _p, _i64, _p]),
    "sv2n_gat_wgrad_node_bf16_workspace": (_i64, [_i64, _i32, _i32, _i32, _i32]),
    "sv2n_gat_wgrad_node_bf16": (_i32, [_p, _i64, _p, _i32, _i64, _i32, _p, _p, _p, _i32, _i32,
                                        _p, _i32, _i32, _p, _p, _p, _p, _p, _i64, _p]),
    "sv2n_gat_wgrad_node_bf16b": (_i32, [_p, _i64, _p, _i64, _i64, _i32, _i32, _p, _p, _p, _i32,
                                         _i32, _p, _i32, _i32, _p, _p, _p, _p, _p, _i64, _p]),
    "sv2n_gat_prep_bwd_node": (_i32, [_p, _i32, _p, _p, _p, _i32, _i32, _i32, _p, _i32, _i32, _p,
                                      _p, _p, _p, _p, _i64, _p]),
    "sv2n_gat_prep_bwd_edge": (_i32, [_p, _i32, _i32, _p, _p, _i32, _i32, _i32, _p, _p, _p]),
    "sv2n_gat_prep_bwd_edge_all": (_i32, [_p, _i32, _i32, _p, _i32, _p]),
    "sv2n_adam_f32": (_i32, [_p, _p, _p, _p, _i64, _p, _f32, _f32, _f32, _f32, _f32, _p]),
    "sv2n_adam_f32_step": (_i32, [_p, _p, _p, _p, _i64, _p, _p, _f32, _f32, _f32, _f32, _f32,
                                  _p]),
    "sv2n_dropout_uniform": (_i32, [_p, _i64, _u64, _p, _u32, _p]),
    "sv2n_edge_logits_fwd_cv": (_i32, [_p, _i64, _i32, _i32, _p, _p, _i32, _p, _i32, _i32, _p]),
    "sv2n_edge_logits_bwd_cv_workspace": (_i64, [_i32, _i32]),
    "sv2n_edge_logits_bwd_cv": (_i32, [_p, _i64, _i32, _i32, _p, _p, _i32, _i32, _p, _i64, _p,
                                       _i32, _p]),
    "sv2n_head_mse_workspace": (_i64, [_i64, _i32, _i32]),
    "sv2n_head_mse_train_workspace": (_i64, [_i64, _i32, _i32]),
    "sv2n_head_mse_train": (_i32, [_p, _i64, _i32, _p, _p, _i32, _p, _p, _p, _p, _p, _p, _p, _i64,
                                   _p]),
    "sv2n_head_mse_train_rows": (_i32, [_p, _i64, _i32, _p, _p, _i32, _p, _p, _p, _i64, _p]),
    "sv2n_head_mse_train_reduce": (_i32, [_p, _i64, _i64, _i32, _i32, _p, _p, _p, _p, _p]),
    "sv2n_head_mse_fwd": (_i32, [_p, _i64, _i32, _p, _p, _i32, _p, _p, _p, _p, _p, _p, _i64, _p]),
    "sv2n_head_mse_bwd": (_i32, [_p, _i64, _i32, _p, _i32, _p, _p, _p, _p, _p, _p, _i64, _p]),
    "sv2n_head_fwd": (_i32, [_p, _i64, _i32, _p, _p, _i32, _p, _p]),
    "sv2n_window_gather": (_i32, [_p, _p, _i32, _i64, _p, _i64, _i64, _i32, _i32, _p, _p, _p, _p,
                                  _p]),
    "sv2n_window_gather_diag": (_i32, [_p, _p, _p, _i32, _i64, _p, _i64, _i64, _i32, _i32, _p, _p,
                                       _p, _p, _p]),
    "sv2n_window_gather_bf16x": (_i32, [_p, _p, _p, _i32, _i64, _p, _i64, _i64, _i32, _i32, _p,
                                        _p, _p, _i64, _p, _p, _p]),
    "sv2n_window_gather_cv": (_i32, [_p, _p, _p, _i32, _i64, _p, _i64, _i64, _i32, _i32, _p,
                                     _p, _p, _i64, _p, _p, _p]),
    "sv2n_head_bwd_workspace": (_i64, [_i64, _i32, _i32]),
    "sv2n_head_bwd": (_i32, [_p, _i64, _i32, _p, _i32, _p, _p, _p, _p, _p, _i64, _p]),
}

EXPORTED_SYMBOLS = tuple(_SIGNATURES)

_lib = None


class NativeLibraryError(RuntimeError):
    pass


def load() -> ctypes.CDLL:
    """Load libsv2n.so once; raise NativeLibraryError if it is absent/stale."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeLibraryError(
            f"{LIB_PATH} not found: build it with `make` (hipcc --offload-arch=gfx950) or "
            "`python -c 'import __graft_entry__ as g; g.build()'`. The SpotV2Net GAT hot path "
            "has no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _SIGNATURES.items():
        fn = getattr(lib, name)  # AttributeError => stale library
        fn.restype = res
        fn.argtypes = args
    if lib.sv2n_abi_version() != ABI_VERSION:
        raise NativeLibraryError(f"libsv2n ABI {lib.sv2n_abi_version()} != expected {ABI_VERSION}")
    _lib = lib
    return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().sv2n_strerror(rc).decode()
        raise RuntimeError(f"{what} failed (code {rc}): {msg}")


def ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def stream_handle(device: torch.device) -> int:
    """The raw hipStream_t of the device's current stream (torch's own accessor:
    under torch.compile a resumed frame can see current_stream() as a generic
    torch.Stream without .cuda_stream)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    return torch._C._cuda_getCurrentRawStream(idx)


def ptr_array(ptrs) -> ctypes.Array:
    arr = (ctypes.c_void_p * len(ptrs))()
    for k, p in enumerate(ptrs):
        arr[k] = p
    return arr


_persistent: dict = {}


def persistent_zeros(tag: str, numel: int, device: torch.device,
                     dtype: torch.dtype = torch.float32) -> torch.Tensor:
    """A zero-initialised device buffer reused across calls (workspaces whose
    ticket counters must start at zero; the kernels leave them zero).  Keyed
    by device and size, so a hipGraph capture (which runs on its own stream)
    reuses the buffer made during warm-up instead of recording a fill.  Ops
    sharing a key must not run concurrently on different streams."""
    dev = torch.device(device)
    key = (tag, int(numel), str(dev), dtype)
    buf = _persistent.get(key)
    if buf is None:
        buf = torch.zeros(max(int(numel), 1), device=dev, dtype=dtype)
        _persistent[key] = buf
    return buf
