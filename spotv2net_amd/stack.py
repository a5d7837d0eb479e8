"""Fused GAT stack: all GATConv layers of a GATModel (or one standalone
GATConv) as ONE autograd node whose forward and backward are sequences of
``torch.ops.sv2n`` operators (library.py; each one C-ABI kernel group).

Forward (reference utils/models.py:145-148 with PyG GATConv inside):
  once       sv2n::gat_prep     W -> [W ; Wᵀatt_src ; Wᵀatt_dst], its bf16 planes, W̃_edge
  once       sv2n::edge_logits  edge_attr · W̃ for every layer (one HBM pass)
  per layer  sv2n::project      xs = x · Waugᵀ  (f32-accurate split MFMA, or bf16)
             sv2n::gat_attn_fwd loops/leaky/softmax/dropout/aggregate/bias/act
             dropout between layers (model-level, torch RNG mask)
Edge-fused mode (32 < n <= 256, narrow edge_attr: the C5 shapes, see
``_use_fused``): no edge pass; sv2n::gat_attn_fused_fwd computes each layer's
edge logits from edge_attr inside the attention, and sv2n::gat_attn_fused_bwd
returns the layer's dW̃ columns directly (no logit / d-logit planes).
Backward, layers in reverse:
  sv2n::gat_attn_bwd  -> d xs, d ae, bias partials
  sv2n::gat_wgrad     -> dWaugᵀ = xᵀ·dxs (split-K) + fold epilogue, ACCUMULATED
  sv2n::project       -> dx = dxs·Waug (if needed)
  then one sv2n::edge_logits_bwd for all layers + sv2n::prep_bwd_edge per layer.

Parameter gradients.  By default the node RETURNS its parameter gradients to
autograd (computed into one zero-initialised flat buffer per backward, one view
per parameter), so ``AccumulateGrad`` fills ``p.grad``: parameter hooks,
``torch.autograd.grad(loss, params)`` and ``DistributedDataParallel`` see them
as with PyG.  Inside ``direct_grad_accumulation()`` (what ``train.TrainStep``
uses, with every ``p.grad`` already a view of its flat gradient buffer) the
kernels accumulate straight into ``p.grad`` and the node returns None for the
parameters: no per-parameter autograd launches in the captured step.
"""
from __future__ import annotations

import contextlib
import os
import threading
from typing import Optional, Sequence

import torch

from . import _lib, library  # noqa: F401  (library registers torch.ops.sv2n)
from .layout import GraphLayout, check_full_edge_attr, cov_var_seq_length
from .library import edge_order, fused_supported
from .ops import ACT_CODES, _aligned, _require_device, relu_mask_fusable, resolve_precision

ACT_RELU = ACT_CODES["relu"]


def _grad_buf(p: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    if p is None or not p.requires_grad:
        return None
    if p.grad is None:
        p.grad = torch.zeros_like(p, memory_format=torch.contiguous_format)
    elif not p.grad.is_contiguous():
        p.grad = p.grad.contiguous()
    return p.grad


HEAD_MAX_IN, HEAD_MAX_OUT = 1024, 16   # sv2n_head_* limits (include/sv2n.h)


def head_fits(in_features: int, out_features: int) -> bool:
    """Whether sv2n_head_* take this head (sv2n_head.hip head_rows_per_block:
    at least 32 staged rows of in_features + 1 floats plus the weights in the
    kernels' 140 KiB dynamic LDS)."""
    if not (0 < in_features <= HEAD_MAX_IN and 0 < out_features <= HEAD_MAX_OUT):
        return False
    return in_features <= 128 or 4 * (32 * (in_features + 1) + out_features * in_features) \
        <= 140 * 1024

_mode = threading.local()


@contextlib.contextmanager
def direct_grad_accumulation():
    """Within this context the fused nodes accumulate parameter gradients
    straight into ``p.grad`` (which must be dense fp32) instead of returning
    them to autograd.  Hooks and ``autograd.grad`` do not see such gradients;
    ``train.TrainStep`` uses it around its (captured) forward."""
    prev = getattr(_mode, "direct", False)
    _mode.direct = True
    try:
        yield
    finally:
        _mode.direct = prev


def _direct_mode() -> bool:
    return getattr(_mode, "direct", False)


def _int64_seed(seed: int) -> int:
    """A 64-bit seed as the signed int64 with the same bit pattern (the
    dispatcher refuses ints >= 2**63 for an ``int`` schema argument)."""
    s = int(seed) & 0xFFFFFFFFFFFFFFFF
    return s - (1 << 64) if s >= (1 << 63) else s


@contextlib.contextmanager
def device_dropout(seed: int, step: torch.Tensor):
    """Within this context the post-layer dropout of the n <= 32 attention
    (utils/models.py:148) draws its uniforms from sv2n::dropout_uniform keyed
    by (``seed``, the device step count ``step``, layer) instead of torch's
    generator, so a captured step holds no torch random op (whose replays
    each launch two generator-state fills).  ``train.TrainStep`` uses it with
    its Adam step counter; outside it every draw is torch.rand.

    ``seed`` may be any 64-bit unsigned value (``torch.initial_seed()``): it
    is folded into the int64 range of the op's schema here and reinterpreted
    as uint64 on the C side."""
    prev = getattr(_mode, "drop_rng", None)
    _mode.drop_rng = (_int64_seed(seed), step)
    try:
        yield
    finally:
        _mode.drop_rng = prev


def _drop_rng_key():
    """(seed, step-tensor pointer) of the active device_dropout context, or
    None (a capture's draws depend on both)."""
    rng = getattr(_mode, "drop_rng", None)
    return None if rng is None else (rng[0], rng[1].data_ptr())


def _post_uniforms(rows: int, cols: int, layer: int, dev) -> torch.Tensor:
    rng = getattr(_mode, "drop_rng", None)
    if rng is None:
        return torch.rand(rows, cols, device=dev)
    return torch.ops.sv2n.dropout_uniform(rows, cols, rng[1], rng[0], layer)


class _GradTargets:
    """Where a fused node's kernels accumulate parameter gradients, and what
    its backward returns for the parameters (see module docstring)."""

    def __init__(self, params, needs, direct: bool, device):
        self.direct = direct
        self.flat: Optional[torch.Tensor] = None  # the one buffer behind every view (not direct)
        self._views = {}
        self._used = set()
        self._order = [id(p) for p in params]
        if direct:
            for p, nd in zip(params, needs):
                if nd:
                    self._views[id(p)] = _grad_buf(p)
            return
        total = sum(p.numel() for p, nd in zip(params, needs) if nd)
        if total == 0:
            return
        flat = torch.zeros(total, device=device, dtype=torch.float32)
        self.flat = flat
        off = 0
        for p, nd in zip(params, needs):
            if nd:
                k = p.numel()
                self._views[id(p)] = flat[off:off + k].view(p.shape)
                off += k

    def __call__(self, p) -> Optional[torch.Tensor]:
        """Gradient buffer of p (None when not needed); marks p as written."""
        if p is None:
            return None
        g = self._views.get(id(p))
        if g is not None:
            self._used.add(id(p))
        return g

    def returned(self) -> tuple:
        if self.direct:
            return (None,) * len(self._order)
        return tuple(self._views.get(i) if i in self._used else None for i in self._order)


def layer_params(conv) -> list:
    ps = [conv.lin_src.weight, conv.att_src, conv.att_dst]
    if conv.lin_edge is not None:
        ps += [conv.lin_edge.weight, conv.att_edge]
    if conv.bias is not None:
        ps.append(conv.bias)
    return ps


def _ldx(conv) -> int:
    return (conv.heads * conv.out_channels + 2 * conv.heads + 3) // 4 * 4


def _hp(L: int, H: int) -> int:
    """Edge-fold column padding: L*H -> 4, 8, 16 or 32 (ops.pad_columns)."""
    for hp in (4, 8, 16, 32):
        if L * H <= hp:
            return hp
    raise ValueError(f"at most 32 (layers x heads) edge-logit columns supported, got {L * H}")


# "auto" (the rule in _use_fused), "on" (whenever the kernels take the shape) or
# "off" (always edge pass + planes): an A/B switch for tests and measurements
EDGE_FUSED = os.environ.get("SV2N_EDGE_FUSED", "auto")
LAST_PATH = {"attention": None,   # which attention path the last forward took (tests)
             "edge_tail": None,   # whether the last backward fused the edge gradient
             "cov_var": None}     # whether the last forward took the covariance-layout passes


def _overlap_edge(training: bool) -> bool:
    """Run the edge-logit pass on a side stream beside the layer-0 projection
    GEMM: inference only (MI355X, C2 B = 512: forward 2.18-2.19 M -> 2.24-2.26
    M graphs/s; in the training step 0.5485 vs 0.5473 ms, within noise)."""
    if FWD_OVERLAP != "auto":
        return FWD_OVERLAP == "on"
    return not training


# "on": the backward runs the work off its critical path on a side stream —
# the weight gradients of layers l > 0 beside layer l's dX GEMM and layer
# l-1's attention backward, and the edge-logit gradient pass (+ its fold)
# beside layer 0's weight gradient — joined before the node returns (inside a
# captured step the fork/join becomes graph edges); "off": one stream;
# "auto" (default): the bf16 mode only.  MI355X, round 6
# (`profiles/r06_bwd_overlap_ab.txt`): C3 (bf16, B = 128) 465 -> 474 K
# windows/s; C2 (f32, B = 512) 1,133-1,140 -> 1,112-1,121 K graphs/s — each
# cross-stream dependency of the replayed graph leaves the GPU idle 5-10 us,
# and the concurrent GEMMs slow each other (L1 dX 26 -> 44 us beside L1 dW).
BWD_OVERLAP = os.environ.get("SV2N_BWD_OVERLAP", "auto")
# "auto": the forward's edge pass beside the layer-0 projection in inference
# only (_overlap_edge); "on" / "off": always / never (A/B switch)
FWD_OVERLAP = os.environ.get("SV2N_FWD_OVERLAP", "auto")


def _overlap_bwd(dev, bf16: bool) -> bool:
    if dev.type != "cuda" or BWD_OVERLAP == "off":
        return False
    if torch.compiler.is_compiling():  # streams stay out of traced graphs
        return False
    return BWD_OVERLAP == "on" or bf16


_SIDE = {}


def _side_stream(dev):
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    if key not in _SIDE:
        _SIDE[key] = torch.cuda.Stream(device=dev)
    return _SIDE[key]


def cov_var_edges_only(convs, n: int, seq_length: int) -> bool:
    """Whether the fused stack reads the edge features of canonical complete
    batches (n nodes, edge_attr in the covariance layout of windows of
    ``seq_length``) only through the covariance-layout edge passes, forward
    and backward — the condition for ``WindowDataset.empty_batch(
    cov_var_only=True)`` (``train.Fit``).  Mirrors ``stack_forward``'s ``cv``
    test, which refuses such a batch on any other path."""
    if COV_VAR_EDGES != "on" or COV_VAR_BWD != "on" or not convs:
        return False
    if any(c.lin_edge is None for c in convs):
        return False
    H = convs[0].heads
    if any(c.heads != H for c in convs):
        return False
    # even seq_length: the k_edge_*_cv2 passes, whose reads sv2n_window_gather_cv covers
    return 2 <= n <= 32 and seq_length <= 64 and seq_length % 2 == 0 and len(convs) * H <= 16


def _use_fused(layout: GraphLayout, convs, D: int, num_edges: int) -> bool:
    """Edge-fused attention (sv2n_attn_fused.hip) instead of edge pass + planes.

    Per layer the fused kernels read edge_attr twice (forward, backward):
    8·D bytes per edge.  The planes path reads it twice for all L layers
    (8·D/L per layer) but writes and re-reads a logit plane and a d-logit
    plane: 16·H bytes per edge and layer.  Fused wins when
    8·D·(1 - 1/L) < 16·H, i.e. D·(L-1) < 2·H·L (C5: D 12, L 3, H 8)."""
    if EDGE_FUSED == "off" or not layout.tiled or num_edges == 0:
        return False
    if layout.kind == "block" and layout.eid is None:
        return False
    L = len(convs)
    H = convs[0].heads
    if not all(fused_supported(layout.n, c.heads, c.out_channels, D) for c in convs):
        return False
    return EDGE_FUSED == "on" or D * (L - 1) < 2 * H * L


def _opt(t: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    return None if t is None or t.numel() == 0 else t


# "on": layer 0's attention backward also computes the edge-logit weight
# gradient wherever the kernel takes the shape; "off" (default): the separate
# MFMA edge-gradient pass.  Round 4, C2 traced step on one MI355X: the fused
# tail made layer 0's backward 28 -> 78-80 us against 52 + 5.7 us for the
# separate pass and its reduce, but the next step's edge forward then misses
# the Infinity Cache (43 -> 48 us): step span 543.0 (on) vs 530.6-539.3 us
# (off, `profiles/r04_c2_edge_ab.txt`).
EDGE_TAIL = os.environ.get("SV2N_EDGE_TAIL", "off")

# "on": edge_attr marked as the reference's covariance layout (layout.mark_cov_var)
# goes through the covariance-layout edge passes; "off": the generic passes
# over every edge row (A/B switch for tests and measurements)
COV_VAR_EDGES = os.environ.get("SV2N_COV_VAR_EDGES", "on")
# the backward's covariance-layout pass (sv2n_edge_logits_bwd_cv); "off": the
# generic edge-gradient pass over every row (A/B switch)
COV_VAR_BWD = os.environ.get("SV2N_COV_VAR_BWD", "on")


def _edge_tail_ok(layout: GraphLayout, convs, ea, hp: int) -> bool:
    """Layer 0's n <= 32 attention backward can carry the edge gradient of
    every layer (sv2n_gat_attn_bwd_edge_supported; equal head counts, the
    other layers' d-logits in edge order)."""
    if EDGE_TAIL != "on" or layout.kind == "block" or ea.dim() != 2:
        return False
    H = convs[0].heads
    if any(c.heads != H for c in convs) or len(convs) * H > hp:
        return False
    from .library import attn_bwd_edge_supported
    return attn_bwd_edge_supported(layout.num_graphs, layout.n, H, convs[0].out_channels,
                                   ea.size(1), hp) and ea.data_ptr() % 16 == 0


class _StackMeta:
    """What the backward needs besides the saved tensors (stack_forward)."""
    __slots__ = ("dims", "bf16", "feid", "kscales", "post_p", "head_dz", "cv")

    def __init__(self, dims, bf16, feid, kscales, post_p=None, head_dz=None, cv=False):
        self.dims, self.bf16, self.feid, self.kscales = dims, bf16, feid, kscales
        # the edge passes read edge_attr in its covariance layout (edge_logits_cv)
        self.cv = cv
        # per layer: the post-layer dropout probability when its draws (not a
        # mask) are saved, i.e. the attention kernels apply it themselves
        self.post_p = post_p or [None] * len(kscales)
        # the output head + MSE ran inside the last layer's forward: the
        # gradient its backward starts from (identity activation)
        self.head_dz = head_dz


# "on": in the bf16 mode, layer 0 (input without gradient) keeps bf16 copies of
# its weight-gradient operands (_bf16_export_ok); "off": fp32 operands rounded
# inside the GEMM (A/B switch for tests and measurements)
BF16_OPERANDS = os.environ.get("SV2N_BF16_OPERANDS", "on")

# "on": the training step fuses GATModel.linear + MSE into the last layer's
# attention forward where the kernel takes the shape (gat_train_head_mse);
# "off": the separate head + loss launch (A/B switch for tests and measurements)
HEAD_FUSE = os.environ.get("SV2N_HEAD_FUSE", "on")


def stack_forward(x, edge_attr, convs, layout: GraphLayout, act: int, post_dropout: float,
                  training: bool, precision: str, need_saved: bool, head=None, x_bf16=None):
    """The fused stack's forward launches (module docstring); returns the
    output, the tensors the backward reads and a ``_StackMeta``.  Capturable:
    no host synchronisation, every buffer from the caching allocator.
    ``head`` = (linear, target, g_weight, g_bias, loss_sum or None): the last layer also runs
    the output head and the MSE loss (sv2n::gat_attn_fwd_head_mse, the caller
    checked ``head_mse_fusable``); the output is then the loss and
    ``meta.head_dz`` the last layer's incoming gradient.  ``x_bf16``: bf16(x)
    from the data builder (data.bf16_twin), read by the bf16 mode's layer-0
    GEMMs instead of rounding x."""
    ops = torch.ops.sv2n
    dev = x.device
    L = len(convs)
    B, n, N = layout.num_graphs, layout.n, layout.num_nodes
    use_edge = edge_attr is not None and all(c.lin_edge is not None for c in convs)
    H = convs[0].heads
    tiled = layout.tiled
    bf16 = precision == "bf16"
    if use_edge and any(c.heads != H for c in convs):
        raise NotImplementedError("fused edge pass needs equal head counts across layers")

    ea = None
    hp = 0
    if use_edge:
        ea = edge_attr.view(-1, 1) if edge_attr.dim() == 1 else edge_attr
        ea = _aligned(ea)
        if ea.size(0) != layout.num_edges:
            raise ValueError("edge_attr rows must match edge_index columns")
        hp = _hp(L, H)

    # 1) weight preparation: every layer's folded Waug, its bf16 split planes
    #    (and the transposed ones the backward's dx GEMM needs) and the edge
    #    fold, in one launch (sv2n::gat_prep)
    # the transposed planes feed the backward's dX GEMMs: whenever a backward
    # may run (need_saved: training, or eval mode with a gradient asked for),
    # not only in training — in bf16 mode Waug is a placeholder the dX GEMM
    # cannot fall back to
    need_t = [bool(need_saved and (l > 0 or x.requires_grad)) for l in range(L)]
    waugs, planes, planes_t, wf = ops.gat_prep(
        [c.lin_src.weight for c in convs], [c.att_src for c in convs],
        [c.att_dst for c in convs], [c.lin_edge.weight for c in convs] if use_edge else [],
        [c.att_edge for c in convs] if use_edge else [], [c.heads for c in convs],
        [c.out_channels for c in convs], hp, need_t, use_edge, bf16)

    # 2) edge logits of every layer in one pass over edge_attr (sv2n::edge_logits),
    #    unless the attention computes them itself (edge-fused mode)
    aes = [None] * L
    ei = layout.edge_index if layout.kind == "block" else None
    # canonical batches: AE in edge order [E][H] (coalesced on both sides)
    eo = bool(use_edge and not tiled and edge_order(ei, n))
    fused = bool(use_edge and _use_fused(layout, convs, ea.size(1), ea.size(0)))
    feid = layout.eid if (fused and layout.kind == "block") else None
    LAST_PATH["attention"] = "fused" if fused else ("tiled" if tiled else "small")
    # edge features the builder wrote in the reference's covariance layout
    # (layout.mark_cov_var): the edge passes read the covariance columns of the
    # upper rows and one variance series per node (sv2n_edge_logits_fwd_cv)
    s_cv = cov_var_seq_length(edge_attr) if use_edge else None
    cv = bool(s_cv is not None and COV_VAR_EDGES == "on" and not fused and not tiled and
              layout.kind == "canonical" and 2 <= n <= 32 and s_cv <= 64 and L * H <= 16 and
              ea.size(1) == 3 * s_cv and ea.size(0) == B * n * (n - 1))
    LAST_PATH["cov_var"] = cv
    if use_edge and not (cv and (COV_VAR_BWD == "on" or not training)):
        check_full_edge_attr(edge_attr, "this model's edge path (not the covariance-layout passes)")

    def edge_fwd():
        if cv:
            return list(ops.edge_logits_cv(ea, wf, layout.canon, L, H, B, n))
        return list(ops.edge_logits(ea, wf, ei, layout.canon, L, H, B, n, tiled))

    overlap = None
    if use_edge and not fused:
        if _overlap_edge(need_saved) and dev.type == "cuda":
            # the edge pass (HBM-bound) on a side stream beside the layer-0
            # projection (MFMA-bound); joined before layer 0's attention
            main = torch.cuda.current_stream(dev)
            side = _side_stream(dev)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                aes = edge_fwd()
            for a in aes:
                a.record_stream(main)
            overlap = (main, side)
        else:
            aes = edge_fwd()
        if tiled and ea.size(0) == 0:
            aes = [None] * L

    # 3) layers
    # x of a twin-only batch (data.twin_only_x) is NaN: only the bf16 twin may
    # be read, by the layer-0 projection and weight-gradient GEMMs
    twin_only = bool(getattr(x, "_sv2n_twin_only", False))
    xin = _aligned(x)
    if twin_only:
        xin._sv2n_twin_only = True
    xb0 = None  # bf16(x) of layer 0 (bf16 mode, x without grad)
    saved_x, saved_xs, saved_y, saved_p, saved_keep, saved_drop = [], [], [], [], [], []
    saved_st = []
    post_p = []
    for l, c in enumerate(convs):
        Hc, C = c.heads, c.out_channels
        F = c.in_channels
        if xin.size(1) != F:
            raise ValueError(f"layer {l}: expected {F} input features, got {xin.size(1)}")
        if l == 0 and bf16 and x_bf16 is not None and _a16_ok(x_bf16, xin, planes[l]):
            # bf16 mode with bf16(x) from the data builder: no rounding pass
            xs = ops.project_a16(x_bf16, F, planes[l], waugs[l])
            if _bf16_export_ok(bf16, training and need_saved and not need_t[0], xin, c,
                               fused or tiled):
                xb0 = x_bf16
        elif l == 0 and _bf16_export_ok(bf16, training and need_saved and not need_t[0], xin, c,
                                        fused or tiled):
            # bf16 mode: the projection also leaves bf16(x) for the layer's
            # weight-gradient GEMM (sv2n_gemm_bf16_export)
            xs, xb0 = ops.project_bf16_export(xin, planes[l], waugs[l])
        elif l == 0 and twin_only:
            raise RuntimeError(_TWIN_ONLY_MSG.format("layer 0's projection (no bf16-twin GEMM "
                                                     "for this model / batch)"))
        else:
            xs = ops.project(xin, planes[l], waugs[l], False, bf16)  # x · Waugᵀ
        if overlap is not None:
            overlap[0].wait_stream(overlap[1])
            overlap = None
        keep, kscale = None, 1.0
        kn = n if tiled else 32  # keep-mask tile: [B][H][n][n] tiled, [B][H][32][32] per-graph
        if training and c.dropout > 0.0:
            if c.dropout >= 1.0:
                keep = torch.zeros(B, Hc, kn, kn, device=dev, dtype=torch.uint8)
                kscale = 0.0
            else:
                keep = (torch.rand(B, Hc, kn, kn, device=dev) >= c.dropout).to(torch.uint8)
                kscale = 1.0 / (1.0 - c.dropout)
        st = None
        if fused:
            # saved: pre-bias head aggregates + per-row softmax statistics
            y, ps, st = ops.gat_attn_fused_fwd(xs, ea, wf, l * H, feid, c.bias, keep, kscale,
                                               B, n, Hc, C, c.concat, act,
                                               float(c.negative_slope), need_saved)
        elif tiled:
            # nothing saved: the backward recomputes the attention from xs and ae
            y = ops.gat_attn_tiled_fwd(xs, aes[l], layout.num_edges, layout.eid,
                                       layout.rowmask, c.bias, keep, kscale, B, n, Hc, C,
                                       c.concat, act, float(c.negative_slope))
            ps = aes[l]
        post_u = None
        if head is not None and l == L - 1:
            lin, target, ghw, ghb, lsum = head
            if training and 0.0 < post_dropout < 1.0:
                post_u = _post_uniforms(N, Hc * C if c.concat else C, l, dev)
            y, ps, out = ops.gat_attn_fwd_head_mse(
                xs, aes[l], layout.rowmask, c.bias, keep, kscale, post_u,
                float(post_dropout) if post_u is not None else 0.0, lin.weight.view(-1), lin.bias,
                target.reshape(-1), ghw, ghb, B, n, Hc, C, c.concat, act,
                float(c.negative_slope), eo, lsum)
            post_u = None  # applied: y is the layer's incoming gradient dz
        elif not (fused or tiled) and training and 0.0 < post_dropout < 1.0:
            # the post-layer dropout (utils/models.py:148) fused into the
            # attention's store: torch draws the uniforms (same stream as
            # rand_like(y) >= p; device_dropout: sv2n::dropout_uniform), the
            # kernel masks, scales and writes both y (for the activation's
            # backward) and the layer output
            post_u = _post_uniforms(N, Hc * C if c.concat else C, l, dev)
            y, ps, out = ops.gat_attn_fwd_post(xs, aes[l], layout.rowmask, c.bias, keep, kscale,
                                               post_u, float(post_dropout), B, n, Hc, C,
                                               c.concat, act, float(c.negative_slope), eo)
        elif not (fused or tiled):
            y, ps = ops.gat_attn_fwd(xs, aes[l], layout.rowmask, c.bias, keep, kscale, B, n,
                                     Hc, C, c.concat, act, float(c.negative_slope), eo)
        head_last = head is not None and l == L - 1
        if post_u is None and not head_last:
            out = y
        dmask = post_u
        post_p.append(float(post_dropout) if post_u is not None else None)
        if post_u is None and training and post_dropout > 0.0 and not head_last:
            if post_dropout >= 1.0:
                dmask = torch.zeros_like(y)
            else:
                dmask = (torch.rand_like(y) >= post_dropout).to(torch.float32) * \
                    (1.0 / (1.0 - post_dropout))
            out = y * dmask
        saved_x.append(xin)
        saved_xs.append(xs)
        saved_y.append(y)
        saved_p.append(ps)
        saved_st.append(st)
        saved_keep.append(keep)
        saved_drop.append(dmask)
        xin = out

    meta = _StackMeta((L, act, use_edge, hp, H, eo, fused), bf16, feid,
                      [(1.0 / (1.0 - c.dropout)) if (training and 0.0 < c.dropout < 1.0) else
                       (0.0 if training and c.dropout >= 1.0 else 1.0) for c in convs], post_p,
                      saved_y[-1] if head is not None else None, cv)
    saved = [ea, wf if fused else None, *saved_x, *saved_xs, *saved_y, *saved_p, *saved_st,
             *saved_keep, *saved_drop, *waugs, *planes_t, xb0]
    return xin, saved, meta


def stack_backward(saved, meta: _StackMeta, convs, layout: GraphLayout, dout, need_x0: bool,
                   grad_of: "_GradTargets"):
    """The fused stack's backward launches, layers in reverse (module
    docstring); parameter gradients go where ``grad_of`` says; returns dx."""
    ops = torch.ops.sv2n
    L, act, use_edge, hp, H, eo, fused = meta.dims
    sv = saved
    ea, wf = sv[0], sv[1]
    k = 2
    xs_in = sv[k:k + L]; k += L
    xss = sv[k:k + L]; k += L
    ys = sv[k:k + L]; k += L
    pss = sv[k:k + L]; k += L
    sts = sv[k:k + L]; k += L
    keeps = sv[k:k + L]; k += L
    drops = sv[k:k + L]; k += L
    waugs = sv[k:k + L]; k += L
    planes_t = sv[k:k + L]; k += L
    xb0 = sv[k]  # bf16(x) of layer 0, or None
    dev = dout.device
    B, n, N = layout.num_graphs, layout.n, layout.num_nodes

    dy = dout.contiguous()
    daes = [None] * L
    dwf = torch.zeros_like(wf) if fused else None  # every layer writes its own columns
    # the activation backward left to layer l's attention backward (none when
    # the fused head's forward already produced the last layer's dZ)
    act_l = 0 if meta.head_dz is not None else act
    # canonical complete graphs: layer 0's attention backward also computes the
    # edge-logit weight gradient of every layer (sv2n_gat_attn_bwd_edge), so
    # edge_attr is streamed there and no separate edge-gradient pass runs
    need_edge = use_edge and ea is not None and ea.size(0) > 0 and any(
        grad_of(c.lin_edge.weight) is not None or grad_of(c.att_edge) is not None for c in convs)
    edge_tail = bool(need_edge and not fused and not layout.tiled and eo and not meta.cv and
                     _edge_tail_ok(layout, convs, ea, hp))
    LAST_PATH["edge_tail"] = edge_tail

    def edge_grads():
        # every layer's edge-logit weight gradient, then the edge folds
        nonlocal dwf
        if not (use_edge and ea is not None):
            return
        # grads exist (zeros) even without edges, as in PyG
        need_e = [(grad_of(c.lin_edge.weight), grad_of(c.att_edge)) for c in convs]
        if ea.size(0) > 0 and any(a is not None or b is not None for a, b in need_e):
            ei = layout.edge_index if layout.kind == "block" else None
            if meta.cv and COV_VAR_BWD == "on":
                dwf = ops.edge_logits_bwd_cv(ea, layout.canon, daes, H, B, n, hp)
            elif not fused and not edge_tail:
                dwf = ops.edge_logits_bwd(ea, ei, layout.canon, daes, H, B, n, hp,
                                          layout.tiled)
            if all(a is not None and b is not None for a, b in need_e):
                # every layer's edge-fold backward in one launch
                ops.prep_bwd_edge_all(dwf, [l * H for l in range(L)],
                                      [c.lin_edge.weight for c in convs],
                                      [c.att_edge for c in convs], [c.heads for c in convs],
                                      [c.out_channels for c in convs],
                                      [a for a, _ in need_e], [b for _, b in need_e])
            else:
                for l, c in enumerate(convs):
                    gWe, gae = need_e[l]
                    ops.prep_bwd_edge(dwf, l * H, c.lin_edge.weight, c.att_edge, c.heads,
                                      c.out_channels, gWe, gae)

    # work off the critical path (BWD_OVERLAP) goes to a side stream: it waits
    # for everything the main stream queued so far, the tensors it reads stay
    # referenced until the join at the end (so the caching allocator cannot
    # hand their memory to a main-stream allocation while the side stream
    # still reads them), and the gradient buffers it writes are only read
    # after the join
    side = _side_stream(dev) if _overlap_bwd(dev, meta.bf16) else None
    main = torch.cuda.current_stream(dev) if side is not None else None
    held = []
    edge_forked = False

    def on_side(fn, *reads):
        side.wait_stream(main)
        held.extend(t for t in reads if t is not None)
        with torch.cuda.stream(side):
            fn()

    def fork_edge():
        # after layer 0's attention backward every d-logit plane exists
        nonlocal edge_forked
        if side is not None and not edge_forked:
            edge_forked = True
            on_side(edge_grads, ea, dwf, *daes)

    for l in range(L - 1, -1, -1):
        c = convs[l]
        Hc, C = c.heads, c.out_channels
        post_u = drops[l] if meta.post_p[l] is not None else None
        if drops[l] is not None and post_u is None:
            dy = dy * drops[l]
        xs = xss[l]
        if fused:  # pss[l], sts[l]: the forward's head aggregates and row statistics
            dxs, dbp = ops.gat_attn_fused_bwd(
                dy, ys[l], pss[l], sts[l], xs, ea, wf, l * H, meta.feid, keeps[l],
                meta.kscales[l], dwf, B, n, Hc, C, c.concat, act, float(c.negative_slope))
            dae = None
        elif layout.tiled:  # pss[l] holds the layer's ae (or None without edges)
            dxs, dae, dbp = ops.gat_attn_tiled_bwd(
                dy, ys[l], xs, pss[l], layout.num_edges, layout.eid, keeps[l],
                meta.kscales[l], layout.rowmask, B, n, Hc, C, c.concat, act,
                float(c.negative_slope))
        elif l == 0 and xb0 is not None and not need_x0 and not edge_tail and \
                grad_of(c.lin_src.weight) is not None:
            # bf16 mode: dxs as bf16 straight from the attention backward, both
            # weight-gradient operands bf16 in memory (the GEMM rounds fp32
            # operands the same way while staging them)
            dxb, dae, dbp = ops.gat_attn_bwd_bf16dx(
                dy, ys[l], xs, pss[l], keeps[l], meta.kscales[l], layout.rowmask, use_edge,
                B, n, Hc, C, c.concat, act_l, float(c.negative_slope), eo, post_u,
                meta.post_p[l] or 0.0)
            daes[l] = _opt(dae)
            fork_edge()
            ops.gat_wgrad_bf16b(xb0, dxb, c.lin_src.weight, c.att_src, c.att_dst, dbp, Hc, C,
                                grad_of(c.lin_src.weight), grad_of(c.att_src),
                                grad_of(c.att_dst), grad_of(c.bias))
            continue  # layer 0 without dx (x needs no gradient): nothing else to do
        elif edge_tail and l == 0:
            dxs, dbp, dwf = ops.gat_attn_bwd_edge(
                dy, ys[l], xs, pss[l], keeps[l], meta.kscales[l], ea,
                [None] + [_opt(d) for d in daes[1:]], 0, hp, B, n, Hc, C, c.concat, act_l,
                float(c.negative_slope), post_u, meta.post_p[l] or 0.0)
            dae = None
        else:
            dxs, dae, dbp = ops.gat_attn_bwd(
                dy, ys[l], xs, pss[l], keeps[l], meta.kscales[l], layout.rowmask, use_edge,
                B, n, Hc, C, c.concat, act_l, float(c.negative_slope), eo, post_u,
                meta.post_p[l] or 0.0)
        daes[l] = _opt(dae)
        if l == 0:
            if getattr(xs_in[0], "_sv2n_twin_only", False):
                raise RuntimeError(_TWIN_ONLY_MSG.format("layer 0's weight gradient (fp32 x)"))
            fork_edge()
        gW = grad_of(c.lin_src.weight)
        gas = grad_of(c.att_src)
        gad = grad_of(c.att_dst)
        gb = grad_of(c.bias)
        if any(g is not None for g in (gW, gas, gad, gb)):
            # split-K dWaugᵀ GEMM + one fused epilogue (fold, transpose,
            # att and bias grads), accumulated into the gradient buffers
            def wgrad(l=l, c=c, dxs=dxs, dbp=dbp, gW=gW, gas=gas, gad=gad, gb=gb):
                ops.gat_wgrad(xs_in[l], dxs, c.lin_src.weight, c.att_src, c.att_dst, dbp, Hc,
                              C, meta.bf16, gW, gas, gad, gb)
            if side is not None and l > 0:
                # off the critical path: layer l's dX GEMM and layer l-1's
                # attention backward run beside it
                on_side(wgrad, xs_in[l], dxs, dbp)
            else:
                wgrad()
        act_l = act
        if l > 0 or need_x0:
            # dxs · Waug; ahead of a ReLU layer on the n <= 32 path the GEMM
            # stores dZ = relu'(y)·dy itself (sv2n_gemm_f32x3_relu) and that
            # layer's attention backward runs with the identity (reads no y)
            relu_y = None
            if l > 0 and act == ACT_RELU and not fused and not layout.tiled and \
                    relu_mask_fusable(dxs, _opt(planes_t[l]), meta.bf16):
                relu_y, act_l = ys[l - 1], 0
            dy = ops.project(dxs, _opt(planes_t[l]), waugs[l], True, meta.bf16, relu_y)

    if not edge_forked:
        edge_grads()
    if side is not None:
        main.wait_stream(side)  # the join: gradients complete on the main stream
        held.clear()
    return dy if need_x0 else None


class _GATStack(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, edge_attr, convs, layout: GraphLayout, act: int, post_dropout: float,
                training: bool, precision: str, x_bf16, *params):
        out, saved, meta = stack_forward(x, edge_attr, convs, layout, act, post_dropout, training,
                                         precision, training or any(ctx.needs_input_grad),
                                         x_bf16=x_bf16)
        ctx.convs = convs
        ctx.layout = layout
        ctx.direct = _direct_mode()
        ctx.meta = meta
        ctx.save_for_backward(*saved)
        return out

    @staticmethod
    def backward(ctx, dout):
        params = [p for c in ctx.convs for p in layer_params(c)]
        grad_of = _GradTargets(params, ctx.needs_input_grad[9:], ctx.direct, dout.device)
        dx0 = stack_backward(ctx.saved_tensors, ctx.meta, ctx.convs, ctx.layout, dout,
                             ctx.needs_input_grad[0], grad_of)
        return (dx0, None, None, None, None, None, None, None, None) + grad_of.returned()


def _a16_ok(x_bf16: torch.Tensor, xin: torch.Tensor, planes) -> bool:
    """sv2n_gemm_bf16_a16 takes the layer-0 projection from the bf16 twin of x
    (its large-tile shapes, 16-B rows of the twin)."""
    return (BF16_OPERANDS == "on" and planes is not None and x_bf16.dtype == torch.bfloat16
            and x_bf16.shape[0] == xin.shape[0] and x_bf16.shape[1] >= xin.shape[1]
            and x_bf16.stride(1) == 1 and x_bf16.stride(0) % 8 == 0
            and x_bf16.data_ptr() % 16 == 0 and xin.shape[0] >= 1024 and planes.shape[-2] >= 384)


_TWIN_ONLY_MSG = ("{} reads x, which this batch holds only as its bf16 twin "
                  "(data.WindowDataset.empty_batch(twin_only=True))")


def twin_only_ok(convs, rows: int) -> bool:
    """Whether layer 0 of this stack reads a ``rows``-node bf16 batch's x
    only through its bf16 twin (``_a16_ok``'s shape conditions, the bf16
    operand path on, a weight that trains): ``train.Fit`` then has the
    gather write the twin alone (data.WindowDataset.empty_batch(twin_only=True)).
    The stack re-checks on the tensors and refuses a twin-only batch on any
    other path."""
    from .library import _ldx
    c = convs[0]
    return (BF16_OPERANDS == "on" and rows >= 1024 and _ldx(c.heads, c.out_channels) >= 384
            and c.lin_src.weight.requires_grad)


def _bf16_export_ok(bf16: bool, want: bool, xin: torch.Tensor, conv, other_path: bool) -> bool:
    """Layer 0 in the bf16 mode whose input needs no gradient: its projection
    exports bf16(x) and its backward runs on bf16 operands end to end
    (sv2n_gemm_bf16_export, sv2n_gat_attn_bwd_bf16dx, sv2n_gat_wgrad_node_bf16b)."""
    return (bf16 and want and BF16_OPERANDS == "on" and not other_path
            and conv.lin_src.weight.requires_grad
            and xin.size(1) % 4 == 0 and xin.stride(1) == 1 and xin.stride(0) % 4 == 0
            and xin.data_ptr() % 16 == 0)


def head_mse_fusable(convs, layout: GraphLayout, linear: torch.nn.Linear,
                     post_dropout: float) -> bool:
    """Whether the training step can run GATModel.linear + MSE inside the last
    layer's attention forward (sv2n_gat_attn_fwd_head_mse_supported: the
    n <= 32 path with one workgroup per graph, out_features 1)."""
    from .library import attn_fwd_head_mse_supported
    last = convs[-1]
    return (HEAD_FUSE == "on" and not layout.tiled and linear.out_features == 1
            and post_dropout < 1.0 and last.in_channels > 0
            and attn_fwd_head_mse_supported(layout.num_graphs, layout.n, last.heads,
                                            last.out_channels, last.concat))


def gat_train_head_mse(x: torch.Tensor, edge_attr: Optional[torch.Tensor], convs: Sequence,
                       layout: GraphLayout, act: int, post_dropout: float, linear: torch.nn.Linear,
                       target: torch.Tensor, precision: Optional[str] = None,
                       x_bf16: Optional[torch.Tensor] = None,
                       loss_sum: Optional[torch.Tensor] = None):
    """One training forward + backward with the upstream loss gradient 1
    (5_train_SpotV2Net.py:150-158: ``loss = MSELoss()(model(data), y);
    loss.backward()``) with the output head and the loss fused into the last
    layer's attention forward: parameter gradients ACCUMULATE into ``p.grad``
    (direct mode, as ``train.TrainStep`` keeps them); returns the loss, or
    None when the shape does not fuse (the caller takes the unfused path).
    No autograd graph is built; capturable."""
    if not head_mse_fusable(convs, layout, linear, post_dropout):
        return None
    precision = resolve_precision(precision)
    params = [p for c in convs for p in layer_params(c)]
    _require_params(params + [linear.weight, linear.bias])
    _require_device(x, edge_attr, target)
    if edge_attr is not None and edge_attr.requires_grad:
        raise NotImplementedError("gradients w.r.t. edge_attr are not supported")
    grad_of = _GradTargets(params, [p.requires_grad for p in params], True, x.device)
    ghw = _grad_buf(linear.weight) if linear.weight.requires_grad else None
    ghb = _grad_buf(linear.bias) if linear.bias is not None and linear.bias.requires_grad \
        else None
    with torch.no_grad():
        loss, saved, meta = stack_forward(x, edge_attr, tuple(convs), layout, int(act),
                                          float(post_dropout), True, precision, True,
                                          head=(linear, target, ghw, ghb, loss_sum),
                                          x_bf16=x_bf16)
        stack_backward(saved, meta, tuple(convs), layout, meta.head_dz, False, grad_of)
        if layout.pending is not None:
            # the kernels added the loss to loss_sum and the gradients to
            # p.grad themselves: carry the deferred edge check's NaN poison
            # into those too (x·1 is exact; one multi-tensor launch), as the
            # unfused path's NaN outputs would
            f = torch.where(layout.pending[0] != 0, float("nan"), 1.0).to(torch.float32)
            bufs = [q.grad for q in params + [linear.weight, linear.bias]
                    if q is not None and q.grad is not None]
            if loss_sum is not None:
                bufs.append(loss_sum)
            torch._foreach_mul_(bufs, f)
    return layout.poison(loss).reshape(())


def _require_params(params) -> None:
    """The kernels read every parameter as a dense fp32 buffer through its raw
    pointer: refuse anything else (stock PyTorch raises a dtype mismatch for
    ``model.double()`` with fp32 data; here it would read garbage)."""
    for p in params:
        if p is None:
            continue
        if p.dtype != torch.float32:
            raise TypeError(f"spotv2net_amd parameters must be float32 (got {p.dtype}); the "
                            "kernels keep fp32 master weights (bf16 is an execution mode, "
                            "see GATModel.set_precision)")
        if not p.is_contiguous():
            raise TypeError("spotv2net_amd parameters must be contiguous")


def gat_stack(x: torch.Tensor, edge_attr: Optional[torch.Tensor], convs: Sequence,
              layout: GraphLayout, act: int, post_dropout: float, training: bool,
              precision: Optional[str] = None,
              x_bf16: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Run ``convs`` (GATConv modules) as one fused autograd node.

    ``precision``: "f32" (f32-accurate GEMMs, 1e-5 parity with PyG fp32) or
    "bf16" (projection and weight-gradient GEMMs on bf16 operands with fp32
    accumulation; softmax, aggregation and edge logits stay fp32); None =
    bf16 inside torch.autocast(cuda, bfloat16), else f32."""
    precision = resolve_precision(precision)
    params = []
    for c in convs:
        params += layer_params(c)
    _require_params(params)
    _require_device(x, edge_attr)
    if edge_attr is not None and edge_attr.requires_grad:
        raise NotImplementedError("gradients w.r.t. edge_attr are not supported (the reference "
                                  "treats edge_attr as data)")
    for p in params:
        if p.device != x.device:
            raise RuntimeError("parameters and data must be on the same device")
    out = _GATStack.apply(x, edge_attr, tuple(convs), layout, int(act), float(post_dropout),
                          bool(training), precision, x_bf16, *params)
    return layout.poison(out)  # NaN if a deferred layout check failed (layout.py)


class _Head(torch.autograd.Function):
    """GATModel.linear (reference utils/models.py:120, :150) on sv2n::head_*;
    parameter gradients are returned (or accumulated directly) like the GAT stack."""

    @staticmethod
    def forward(ctx, x, linear, weight, bias):
        x = _aligned(x)
        out = torch.ops.sv2n.head_fwd(x, weight, bias)
        ctx.linear = linear
        ctx.direct = _direct_mode()
        ctx.save_for_backward(x)
        return out

    @staticmethod
    def backward(ctx, dout):
        (x,) = ctx.saved_tensors
        lin = ctx.linear
        grad_of = _GradTargets([lin.weight, lin.bias], ctx.needs_input_grad[2:4], ctx.direct,
                               x.device)
        dx = torch.ops.sv2n.head_bwd(x, lin.weight, dout, grad_of(lin.weight), grad_of(lin.bias))
        return (dx if ctx.needs_input_grad[0] else None, None) + grad_of.returned()


class _HeadMSE(torch.autograd.Function):
    """``F.mse_loss(linear(x).view(-1), target)`` (reference
    5_train_SpotV2Net.py:150-154) as two launches: sv2n::head_mse_fwd (head,
    residual, loss) and sv2n::head_mse_bwd (dx and the head's parameter grads)."""

    @staticmethod
    def forward(ctx, x, target, linear, weight, bias, loss_sum=None):
        x = _aligned(x)
        loss, diff = torch.ops.sv2n.head_mse_fwd(x, weight, bias, target, loss_sum)
        ctx.linear = linear
        ctx.direct = _direct_mode()
        ctx.save_for_backward(x, diff)
        return loss

    @staticmethod
    def backward(ctx, gloss):
        x, diff = ctx.saved_tensors
        lin = ctx.linear
        grad_of = _GradTargets([lin.weight, lin.bias], ctx.needs_input_grad[3:5], ctx.direct,
                               x.device)
        dx = torch.ops.sv2n.head_mse_bwd(x, lin.weight, diff, gloss, grad_of(lin.weight),
                                         grad_of(lin.bias))
        return (dx if ctx.needs_input_grad[0] else None, None, None) + grad_of.returned() + \
            (None,)


def head_mse_loss(x: torch.Tensor, linear: torch.nn.Linear, target: torch.Tensor,
                  loss_sum: Optional[torch.Tensor] = None) -> torch.Tensor:
    """mean((linear(x).view(-1) - target)²) with the head and the loss fused.
    ``loss_sum`` (a float32 device scalar): the loss is also added to it in
    the same launch."""
    _require_params((linear.weight, linear.bias))
    _require_device(x, target)
    if not head_fits(linear.in_features, linear.out_features):
        loss = torch.nn.functional.mse_loss(linear(x).view(-1), target)
        if loss_sum is not None:
            loss_sum.add_(loss.detach())
        return loss
    return _HeadMSE.apply(x, target, linear, linear.weight, linear.bias, loss_sum)


def head_mse_train(x: torch.Tensor, linear: torch.nn.Linear, target: torch.Tensor,
                   loss_sum: Optional[torch.Tensor] = None):
    """Training step's head + loss with the upstream loss gradient 1 (what
    ``loss.backward()`` gives): ONE launch returns ``(loss, dx)`` and
    accumulates ``linear``'s parameter gradients into their ``.grad`` — the
    caller continues the backward with ``torch.autograd.backward(x, dx)``.
    Outside autograd; ``train.TrainStep`` uses it (``None`` when the head does
    not fit the kernels)."""
    _require_params((linear.weight, linear.bias))
    _require_device(x, target)
    if not head_fits(linear.in_features, linear.out_features):
        return None
    gw = _grad_buf(linear.weight)
    gb = _grad_buf(linear.bias) if linear.bias is not None else None
    return torch.ops.sv2n.head_mse_train(_aligned(x.detach()), linear.weight.detach(),
                                         None if linear.bias is None else linear.bias.detach(),
                                         target, gw, gb, loss_sum)


def head_mse_train_split(x: torch.Tensor, linear: torch.nn.Linear, target: torch.Tensor,
                         loss_sum: Optional[torch.Tensor] = None):
    """``head_mse_train`` in two launches: dx and the per-block partials now,
    their reduction into the loss, ``loss_sum`` and the head's parameter
    gradients when the caller runs ``finish()`` (``train.TrainStep``: after
    the layer backwards, which need only dx).  The one-launch kernel's
    two-level ticket chain sits between dx and the backward; the separate
    reduce launch does not (C3 loop 433-437 K -> 439-443 K windows/s; running
    it on a side stream beside the backward instead cost the hipGraph's
    fork/join more than it saved: 421-423 K).  Returns ``(loss, dx, finish)``,
    bitwise ``head_mse_train``'s results once ``finish`` ran; ``None`` when
    the head does not fit the wave-per-rows kernel."""
    _require_params((linear.weight, linear.bias))
    _require_device(x, target)
    if not (head_fits(linear.in_features, linear.out_features) and
            library.head_split_fits(linear.in_features, linear.out_features)):
        return None
    gw = _grad_buf(linear.weight)
    gb = _grad_buf(linear.bias) if linear.bias is not None else None
    xa = _aligned(x.detach())
    N, C = xa.shape
    O = linear.out_features
    ws = library.head_split_workspace(N, C, O, xa.device)
    dx = torch.ops.sv2n.head_mse_train_rows(
        xa, linear.weight.detach(), None if linear.bias is None else linear.bias.detach(),
        target, ws)
    loss = torch.empty((), device=xa.device)

    def finish() -> None:
        torch.ops.sv2n.head_mse_train_reduce(ws, N, C, O, loss, gw, gb, loss_sum)

    return loss, dx, finish


def linear_head(x: torch.Tensor, linear: torch.nn.Linear) -> torch.Tensor:
    """``linear(x)`` for GATModel's output layer on the sv2n head kernels
    (in_features <= 1024, out_features <= 16; otherwise the nn.Linear itself)."""
    _require_params((linear.weight, linear.bias))
    _require_device(x)
    if not head_fits(linear.in_features, linear.out_features):
        return linear(x)
    return _Head.apply(x, linear, linear.weight, linear.bias)
