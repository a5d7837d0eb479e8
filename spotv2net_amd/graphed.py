"""Per-shape hipGraph replay of ``GATModel.forward`` and its backward, for the
reference's own training loop left unchanged (5_train_SpotV2Net.py:142-160:
a new batch per step, ``model(data)``, ``nn.MSELoss``, ``zero_grad``,
``loss.backward()``, ``torch.optim.Adam.step()``, ``loss.item()``).

Eagerly, every step issues ~25 kernel launches through the operator layer;
the host needs longer to issue them than the GPU needs to run them
(MI355X, C2 B = 512: ~440 µs of host time for the forward, ~600 for the
backward, against ~550 µs of GPU work for the whole step).  Here the second
call with an identical signature captures the model's forward (GAT stack +
output head) into one hipGraph, its first backward captures the backward
(head, GAT stack, every parameter gradient) into another, and later calls
replay them: one launch each way.

The signature (the cache key built in ``forward``) pins everything a replay reads by address or shape:
the device pointers, shapes and strides of ``x`` / ``edge_attr`` and of every
parameter, the graph layout's kind and sizes, train/eval mode, dropout rates,
precision, autograd state.  Inputs are read IN PLACE through their pointers
(nothing is copied): a batch whose tensors sit at the captured addresses with
the captured shapes holds exactly the data the replay should read.  The
per-batch layout tensors of a freshly analysed edge_index (row mask, edge
ids, the deferred-check word, the edge_index itself on the block path) are
copied into the graph's own buffers before each replay.

Autograd semantics are kept: the forward returns a fresh output tensor, the
backward returns fresh gradient tensors (``AccumulateGrad`` fills ``p.grad``
as with the eager path; hooks and ``autograd.grad`` see them).  While a
replayed forward still awaits its backward, a further forward with the same
signature runs eagerly rather than overwrite the saved tensors; a backward
whose saved tensors were overwritten anyway (``retain_graph`` and a second
backward after another forward) raises instead of returning wrong gradients.
``GATModel.graph_replay = False`` turns all of this off.
"""
from __future__ import annotations

import contextlib
import gc
import weakref
from collections import OrderedDict
from typing import Optional

import torch

from .layout import GraphLayout, cov_var_seq_length
from .ops import _aligned, resolve_precision
from .stack import (_GradTargets, _direct_mode, _require_params, head_fits, layer_params,
                    stack_backward, stack_forward)

MAX_ENTRIES = 4      # graphs kept per model (least recently used dropped)
CAPTURE_AFTER = 2    # the n-th call with one signature captures (earlier ones warm up)


@contextlib.contextmanager
def _no_gc():
    """No garbage collection while a capture is open: a collected object may
    release device resources (a dead graph, an event), which a stream capture
    does not permit.  torch.cuda.graph collects once right before capturing."""
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()


def _tsig(t: Optional[torch.Tensor]):
    if t is None:
        return None
    return (t.data_ptr(), tuple(t.shape), tuple(t.stride()), t.dtype)


def _switches():
    """The process-wide path switches a capture bakes in (stack's A/B
    switches) and whether the forward draws its dropout from the device
    generator (stack.device_dropout, keyed on a step count): flipping one
    must capture again, not replay the old variant."""
    from . import stack
    return (stack.COV_VAR_EDGES, stack.COV_VAR_BWD, stack.HEAD_FUSE, stack.BF16_OPERANDS,
            stack.EDGE_FUSED, stack.EDGE_TAIL, stack._drop_rng_key())


def _layout_sig(lay: GraphLayout):
    def shp(t):
        return None if t is None else (tuple(t.shape), t.dtype)
    return (lay.kind, lay.n, lay.num_graphs, lay.num_nodes, lay.num_edges,
            shp(lay.edge_index), shp(lay.rowmask), _tsig(lay.canon), shp(lay.eid),
            shp(lay.pending))


class _Entry:
    """One captured signature: its graphs, static buffers and saved state."""

    def __init__(self, model, layout: GraphLayout, train_graph: bool):
        # weak: the model owns its cache; a cycle would leave dead graphs for
        # the garbage collector, which may then run inside a later capture
        self._model = weakref.ref(model)
        self.train_graph = train_graph
        self.g_fwd: Optional[torch.cuda.CUDAGraph] = None
        self.g_bwd: Optional[torch.cuda.CUDAGraph] = None
        self.gen = 0
        self.ctx_ref = None          # weakref to the autograd node of the last replay
        self.backwarded = True
        # private copies of the per-batch layout tensors (block layouts)
        def cl(t):
            return None if t is None else t.clone()
        self.layout = GraphLayout(layout.kind, layout.n, layout.num_graphs, layout.num_nodes,
                                  layout.num_edges, cl(layout.edge_index), cl(layout.rowmask),
                                  layout.canon, cl(layout.eid), cl(layout.pending))

    @property
    def model(self):
        m = self._model()
        if m is None:
            raise RuntimeError("spotv2net_amd: the model of this graph replay was freed")
        return m

    def load_layout(self, lay: GraphLayout) -> None:
        for mine, new in ((self.layout.edge_index, lay.edge_index),
                          (self.layout.rowmask, lay.rowmask), (self.layout.eid, lay.eid),
                          (self.layout.pending, lay.pending)):
            if mine is not None and mine.data_ptr() != new.data_ptr():
                mine.copy_(new)

    def busy(self) -> bool:
        """A replayed forward whose backward has not run and whose autograd
        graph is still alive: its saved tensors must not be overwritten."""
        return not self.backwarded and self.ctx_ref is not None and self.ctx_ref() is not None

    # -- capture -------------------------------------------------------------
    def capture_fwd(self, x, edge_attr, precision: str) -> None:
        m = self.model
        convs = tuple(m.gat_layers)
        training = m.training
        need_saved = training or self.train_graph
        lay = self.layout
        g = torch.cuda.CUDAGraph()
        # no autograd recording inside the capture (the replay node is the
        # autograd node): the sv2n ops would otherwise grow fallback nodes
        with torch.no_grad(), _no_gc(), torch.cuda.graph(g, capture_error_mode="thread_local"):
            h, saved, meta = stack_forward(x, edge_attr, convs, lay, m._act_code,
                                           float(m.dropout or 0.0), training, precision,
                                           need_saved)
            h = lay.poison(h)
            hx = _aligned(h)
            out = torch.ops.sv2n.head_fwd(hx, m.linear.weight, m.linear.bias)
        self.g_fwd = g
        self.out = out
        if self.train_graph:
            self.hx, self.saved, self.meta = hx, saved, meta
            self.dout = torch.empty_like(out)

    def capture_bwd(self) -> None:
        m = self.model
        convs = tuple(m.gat_layers)
        lin = m.linear
        params = self.params()
        lay = self.layout
        g = torch.cuda.CUDAGraph()
        with torch.no_grad(), _no_gc(), torch.cuda.graph(g, pool=self.g_fwd.pool(),
                                                         capture_error_mode="thread_local"):
            grad_of = _GradTargets(params, [p.requires_grad for p in params], False,
                                   self.out.device)
            dh = torch.ops.sv2n.head_bwd(self.hx, lin.weight, self.dout, grad_of(lin.weight),
                                         grad_of(lin.bias))
            if lay.pending is not None:  # backward of GraphLayout.poison
                dh = torch.where(lay.pending != 0, torch.zeros_like(dh), dh)
            stack_backward(self.saved, self.meta, convs, lay, dh, False, grad_of)
        self.g_bwd = g
        self.grad_flat = grad_of.flat
        # the flat buffer holds the needed gradients back to back, in
        # parameter order (_GradTargets); written ones are returned as views
        # of a fresh copy, the others as None
        self.grad_sizes, self.grad_shapes = [], []  # shape: (slot?, returned?, shape)
        for p in params:
            v = grad_of._views.get(id(p))
            if v is not None:
                self.grad_sizes.append(p.numel())
            self.grad_shapes.append((v is not None, v is not None and id(p) in grad_of._used,
                                     tuple(p.shape)))

    def params(self):
        return _params(self.model)


class _Replay(torch.autograd.Function):
    """Forward = one graph replay; backward = one graph replay + one copy of
    the flat gradient buffer (fresh tensors for AccumulateGrad)."""

    @staticmethod
    def forward(ctx, entry: _Entry, layout: GraphLayout, inputs, *params):
        # the caller has already replayed entry.g_fwd (see forward below)
        entry.gen += 1
        entry.backwarded = False
        ctx.entry, ctx.gen = entry, entry.gen
        # the backward graph reads x / edge_attr in place (layer 0's weight
        # gradient, the edge-gradient pass): hold them until backward, as the
        # eager node's saved tensors do, and remember their versions so an
        # in-place write in between raises as it would eagerly
        ctx.inputs = inputs
        ctx.versions = tuple(t._version for t in inputs)
        entry.ctx_ref = weakref.ref(ctx)
        return entry.out.clone()

    @staticmethod
    def backward(ctx, dout):
        entry: _Entry = ctx.entry
        if ctx.gen != entry.gen:
            raise RuntimeError(
                "spotv2net_amd: the graph-replayed forward this backward belongs to was "
                "overwritten by a later forward (retain_graph with interleaved forwards); set "
                "model.graph_replay = False for this pattern")
        for t, v in zip(ctx.inputs, ctx.versions):
            if t._version != v:
                raise RuntimeError(
                    "spotv2net_amd: one of the variables needed for gradient computation has "
                    f"been modified by an inplace operation (input version {t._version}, "
                    f"expected {v})")
        entry.dout.copy_(dout.reshape(entry.dout.shape))
        if entry.g_bwd is None:
            entry.capture_bwd()
        entry.g_bwd.replay()
        entry.backwarded = True
        parts = iter(entry.grad_flat.clone().split_with_sizes(entry.grad_sizes))
        grads = []
        for slot, used, shape in entry.grad_shapes:
            g = next(parts) if slot else None
            grads.append(g.view(shape) if used else None)
        return (None, None, None) + tuple(grads)


class GraphCache:
    """The captured signatures of one GATModel (at most MAX_ENTRIES)."""

    def __init__(self):
        self.entries: "OrderedDict[tuple, _Entry]" = OrderedDict()
        self.seen: dict = {}

    def clear(self) -> None:
        self.entries.clear()
        self.seen.clear()

    # captured graphs belong to one model instance: copies start empty
    def __deepcopy__(self, memo):
        return GraphCache()

    def __reduce__(self):
        return (GraphCache, ())


def _eligible(model, x, edge_attr) -> bool:
    if torch.compiler.is_compiling() or torch.jit.is_scripting():
        return False
    if not x.is_cuda or torch.cuda.is_current_stream_capturing() or _direct_mode():
        return False
    if model.standardize or x.requires_grad or x.dtype != torch.float32:
        return False
    if edge_attr is not None and (edge_attr.requires_grad or not edge_attr.is_cuda):
        return False
    lin = model.linear
    return head_fits(lin.in_features, lin.out_features)


# Bumped whenever any module registers a parameter or a submodule (attribute
# assignment of an nn.Parameter / nn.Module goes through these hooks), so a
# model's cached parameter list is rebuilt after a replacement.  Walking the
# modules costs ~15-30 µs of nn.Module attribute lookups per call, host time
# the GPU waits through at the start of a synchronised step.
_PARAM_GEN = [0]


def _bump_param_gen(*_):
    _PARAM_GEN[0] += 1


torch.nn.modules.module.register_module_parameter_registration_hook(_bump_param_gen)
torch.nn.modules.module.register_module_module_registration_hook(_bump_param_gen)


def _optional_slots(model) -> tuple:
    """(parameter dict, the bias it held) of the head and of every layer.
    ``module.bias = None`` goes through ``register_parameter(name, None)``,
    which calls no registration hook, so the cached list also checks these
    slots by identity (a stale list would replay a graph that still adds the
    removed bias)."""
    mods = [model.linear, *model.gat_layers]
    return tuple((m._parameters, m._parameters.get("bias")) for m in mods)


def _params(model) -> list:
    c = model.__dict__.get("_sv2n_params")
    if c is not None and c[0] == _PARAM_GEN[0] and all(d.get("bias") is b for d, b in c[2]):
        return c[1]
    ps = [p for c in model.gat_layers for p in layer_params(c)] + \
        [model.linear.weight] + ([model.linear.bias] if model.linear.bias is not None else [])
    model.__dict__["_sv2n_params"] = (_PARAM_GEN[0], ps, _optional_slots(model))
    return ps


def _convs(model) -> tuple:
    """model.gat_layers as a tuple, cached like the parameter list."""
    c = model.__dict__.get("_sv2n_convs")
    if c is not None and c[0] == _PARAM_GEN[0]:
        return c[1]
    convs = tuple(model.gat_layers)
    model.__dict__["_sv2n_convs"] = (_PARAM_GEN[0], convs)
    return convs


def forward(model, data, x, edge_index, edge_attr, layout: GraphLayout) -> Optional[torch.Tensor]:
    """``linear(gat_stack(...))`` of ``model`` on ``data`` as a graph replay,
    or None when the eager path should run (not eligible, or a call that
    warms up / would overwrite a replay still awaiting its backward).
    Everything up to the replay is host work the GPU waits for at the start
    of a synchronised step, so the signature is kept cheap: parameter
    pointers and autograd flags only (a parameter's shape or dtype cannot
    change without its pointer changing)."""
    if not _eligible(model, x, edge_attr):
        return None
    cache: GraphCache = model._graph_cache
    ps = _params(model)
    needs = tuple(p.requires_grad for p in ps)
    train_graph = torch.is_grad_enabled() and any(needs)
    precision = resolve_precision(model.precision)
    key = (model.training, train_graph, precision, torch.is_autocast_enabled("cuda"),
           model._act_code, model.dropout, tuple(c.dropout for c in _convs(model)),
           _tsig(x), _tsig(edge_attr), cov_var_seq_length(edge_attr), _layout_sig(layout), needs,
           tuple([p.data_ptr() for p in ps]), _switches())
    entry = cache.entries.get(key)
    if entry is None:
        k = cache.seen.get(key, 0) + 1
        if len(cache.seen) > 64:
            cache.seen.clear()
        cache.seen[key] = k
        if k < CAPTURE_AFTER:
            return None
        _require_params(ps)
        entry = _Entry(model, layout, train_graph)
        entry.load_layout(layout)
        entry.capture_fwd(x, edge_attr, precision)
        cache.entries[key] = entry
        while len(cache.entries) > MAX_ENTRIES:
            cache.entries.popitem(last=False)
    else:
        cache.entries.move_to_end(key)
    if not train_graph:
        entry.load_layout(layout)
        entry.g_fwd.replay()
        return entry.out.clone()
    if entry.busy():
        return None
    # replay first, then the autograd bookkeeping: Function.apply's argument
    # processing is host time the GPU would otherwise wait through at the start
    # of a synchronised step (the reference loop's loss.item() drains it)
    entry.load_layout(layout)
    entry.g_fwd.replay()
    inputs = (x,) if edge_attr is None else (x, edge_attr)
    return _Replay.apply(entry, layout, inputs, *ps)
