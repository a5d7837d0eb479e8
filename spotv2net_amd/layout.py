"""Graph-batch layout analysis for the dense-block GAT kernels.

The reference feeds GATConv a PyG ``Batch`` of B fully connected n-node graphs
(``CovarianceLaggedDataset``, reference utils/dataset.py:212-226, batched by the
PyG DataLoader at 5_train_SpotV2Net.py:90-91).  The kernels work on that
structure directly: every target's incoming edges live inside its own n-node
block, so per-target softmax/aggregation is a row of an n x n matrix.

``analyze_edge_index`` classifies an ``edge_index`` once and caches the result
on the tensor object (keyed by its version counter):

* ``canonical`` — exactly the reference's edge order for every graph (the
  n(n-1)/2 row-major upper pairs, then the swapped pairs); kernels derive
  (graph, target, source) from the edge id and never read edge_index.
* ``block``     — any order / subset of edges that stay inside n-node blocks
  with no duplicate (source, target) pair; kernels read edge_index, and a
  per-target source bitmask covers absent edges.

Blocks of n <= 32 nodes run on the one-workgroup-per-graph attention
kernels; 32 < n <= 256 (the C5 stress shapes) on the target-row-tiled ones.
Anything else (ragged graph sizes, duplicate edges, n > 256) raises
``UnsupportedLayout``.

Host synchronisation.  ``canonical_edge_index`` tensors (what the window
builders emit) carry their layout: no analysis at all.  When the caller knows
the graph size (``n``: a Batch's ``nodes_per_graph``, or N / ``num_graphs``),
a new edge_index is analysed WITHOUT a host round trip — the reference loop
builds a new PyG Batch every step (5_train_SpotV2Net.py:142-143) and would
otherwise stall the stream once per batch: it takes the block path (valid for
any edge order) and one kernel (sv2n_block_rowmask_checked) builds the row
mask while counting the edges the kernels cannot take.  That count is a
DEFERRED error: the forward's output is poisoned with NaN when it is non-zero
(``GraphLayout.poison``) and the next analysis (or ``check_pending()``)
raises ``UnsupportedLayout`` for it.  Without a size hint the analysis finds
the block size on the device and synchronises once per new edge_index.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch

from . import _lib

MAX_N = 256          # largest block (include/sv2n.h SV2N_MAX_N_TILED)
SMALL_N = 32         # blocks up to this size use the per-graph kernels


class UnsupportedLayout(NotImplementedError):
    pass


@dataclass(frozen=True)
class GraphLayout:
    kind: str                 # 'canonical' | 'block'
    n: int                    # nodes per graph
    num_graphs: int
    num_nodes: int
    num_edges: int
    edge_index: Optional[torch.Tensor]  # read by kernels on the 'block' path
    rowmask: Optional[torch.Tensor]     # int32 [N][ceil(n/32)] source bitmask; None = complete
    canon: Optional[torch.Tensor]       # int16 [n(n-1)] (target<<8 | source) table
    eid: Optional[torch.Tensor] = None  # int32 [N][n] edge ids (tiled 'block' layouts only)
    pending: Optional[torch.Tensor] = None  # int32 [1] device count of invalid edges (deferred)

    def poison(self, out: torch.Tensor) -> torch.Tensor:
        """``out`` with NaN everywhere if the deferred validation found invalid
        edges (device-side select: no host synchronisation)."""
        if self.pending is None:
            return out
        return torch.where(self.pending != 0, torch.full_like(out, float("nan")), out)

    @property
    def tiled(self) -> bool:
        """True when the blocks need the target-row-tiled attention kernels."""
        return self.n > SMALL_N

    @property
    def device(self) -> torch.device:
        t = self.canon if self.canon is not None else self.edge_index
        return t.device


def canonical_pairs(n: int) -> tuple[list[int], list[int]]:
    """(source, target) lists of one graph, in the order of reference
    utils/dataset.py:216-226: np.argwhere(triu(ones, k=1)) row-major pairs
    (u, v) as source u -> target v, then the same pairs swapped."""
    up_s, up_t = [], []
    for u in range(n):
        for v in range(u + 1, n):
            up_s.append(u)
            up_t.append(v)
    return up_s + up_t, up_t + up_s


_canon_cache: dict = {}


def mark_cov_var_only(edge_attr: torch.Tensor) -> torch.Tensor:
    """Record that ``edge_attr`` holds only the columns the covariance-layout
    edge passes read (sv2n_window_gather_cv: the covariance columns of the
    upper rows and one variance series per node); the rest is unwritten.  The
    flag is permanent (not tied to the tensor's version): the fused stack
    refuses such a tensor on any other edge path, and so does GATModel's
    edge BatchNorm (``check_full_edge_attr``)."""
    edge_attr._sv2n_cov_var_only = True
    return edge_attr


def check_full_edge_attr(edge_attr: Optional[torch.Tensor], what: str) -> None:
    """Raise when ``edge_attr`` is a ``mark_cov_var_only`` buffer."""
    if edge_attr is not None and getattr(edge_attr, "_sv2n_cov_var_only", False):
        raise RuntimeError(
            f"sv2n: {what} reads all of edge_attr, but this batch holds only the columns "
            "of the covariance-layout edge passes (WindowDataset.empty_batch(cov_var_only=True))")


def mark_cov_var(edge_attr: Optional[torch.Tensor], seq_length: int):
    """Record that ``edge_attr`` holds edge features in the reference's
    covariance layout (utils/dataset.py:228-243, :279-282: row s -> t is
    [cov_t(s,t) | var_t(s) | var_t(t)], cov the same in both directions, var a
    per-node series) for canonical complete graphs — stated by the builders
    that write it (``window_batch``, ``WindowDataset``).  The edge passes then
    read ≈ 1/6 of it (sv2n_edge_logits_fwd_cv / _bwd_cv).  The mark holds for
    the tensor's current version: an in-place write drops it."""
    if edge_attr is not None and edge_attr.dim() == 2 and edge_attr.size(1) == 3 * seq_length:
        edge_attr._sv2n_cov_var = (int(seq_length), edge_attr._version)
    return edge_attr


def cov_var_seq_length(edge_attr: Optional[torch.Tensor]) -> Optional[int]:
    """seq_length of a ``mark_cov_var`` tensor whose contents are unchanged since."""
    m = getattr(edge_attr, "_sv2n_cov_var", None)
    if m is None or m[1] != edge_attr._version:
        return None
    return m[0]


def canonical_table(n: int, device: torch.device) -> torch.Tensor:
    key = ("table", n, str(device))
    if key not in _canon_cache:
        s, t = canonical_pairs(n)
        vals = [(ti << 8) | si for si, ti in zip(s, t)]
        _canon_cache[key] = torch.tensor(vals, dtype=torch.int32).to(torch.int16).to(device)
    return _canon_cache[key]


def canonical_edge_index(n: int, num_graphs: int = 1, device=None) -> torch.Tensor:
    """Batched canonical edge_index [2, B*n(n-1)] with PyG Batch node offsets.
    The tensor carries its (canonical) layout, so models never analyse it."""
    device = torch.device(device) if device is not None else torch.device("cpu")
    key = ("ei", n, num_graphs, str(device))
    if key not in _canon_cache:
        s, t = canonical_pairs(n)
        one = torch.tensor([s, t], dtype=torch.long)
        off = (torch.arange(num_graphs, dtype=torch.long) * n).repeat_interleave(len(s))
        ei = one.repeat(1, num_graphs) + off.unsqueeze(0)
        ei = ei.to(device)
        if 1 <= n <= MAX_N:
            N = n * num_graphs
            lay = GraphLayout("canonical", n, num_graphs, N, ei.size(1), None, None,
                              canonical_table(n, device))
            for hint in (None, n):
                _attach(ei, (N, hint), lay)
        if num_graphs * len(s) > 10_000_000:
            return ei  # do not pin very large batches in the cache
        _canon_cache[key] = ei
    return _canon_cache[key]


def _words(n: int) -> int:
    return (n + 31) // 32


def _attach(edge_index: torch.Tensor, key, layout: GraphLayout) -> GraphLayout:
    try:
        cache = getattr(edge_index, "_sv2n_layouts", None)
        if cache is None:
            cache = {}
            edge_index._sv2n_layouts = cache
        cache[key] = (edge_index._version, layout)
    except (AttributeError, RuntimeError):
        pass
    return layout


def _cached(edge_index: torch.Tensor, key) -> Optional[GraphLayout]:
    cache = getattr(edge_index, "_sv2n_layouts", None)
    if cache is None or key not in cache:
        return None
    ver, lay = cache[key]
    return lay if ver == edge_index._version else None


# deferred validations: (pinned host count, event, what) of layouts analysed
# without a host synchronisation; checked at the next analysis / check_pending()
_pending: list = []


def check_pending(block: bool = False) -> None:
    """Raise UnsupportedLayout for any earlier sync-free analysis whose device
    check found invalid edges.  ``block`` waits for checks still in flight."""
    keep = []
    err = None
    for host, ev, what in _pending:
        if block:
            ev.synchronize()
        elif not ev.query():  # still in flight: look again next time
            keep.append((host, ev, what))
            continue
        if int(host[0]) != 0 and err is None:
            err = UnsupportedLayout(
                f"{what}: {int(host[0])} edge(s) outside the node range, across n-node blocks "
                "or repeated; the affected forward returned NaN")
    _pending[:] = keep
    if err is not None:
        raise err


def _analyze_deferred(edge_index: torch.Tensor, N: int, n: int, key) -> GraphLayout:
    """Block-path layout with no host synchronisation (module docstring)."""
    device = edge_index.device
    if N % n != 0:
        raise UnsupportedLayout(f"{N} nodes are not a union of {n}-node graphs")
    if n > MAX_N:
        raise UnsupportedLayout(f"graphs of {n} > {MAX_N} nodes")
    E = edge_index.size(1)
    B = N // n
    if E > 0x7FFFFFFF:
        raise UnsupportedLayout("more than 2^31 edges in one batch")
    lib = _lib.load()
    st = _lib.stream_handle(device)
    ei = edge_index.contiguous()
    rowmask = torch.zeros(N * _words(n), dtype=torch.int32, device=device)
    bad = torch.zeros(1, dtype=torch.int32, device=device)
    if E > 0:
        _lib.check(lib.sv2n_block_rowmask_checked(ei.data_ptr(), E, N, n, rowmask.data_ptr(),
                                                  bad.data_ptr(), st), "sv2n_block_rowmask")
    eid = None
    if n > SMALL_N:
        eid = torch.full((N * n,), -1, dtype=torch.int32, device=device)
        if E > 0:
            _lib.check(lib.sv2n_block_eid(ei.data_ptr(), E, N, n, eid.data_ptr(), st),
                       "sv2n_block_eid")
    if not torch.cuda.is_current_stream_capturing():
        host = torch.empty(1, dtype=torch.int32, pin_memory=True)
        host.copy_(bad, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(device))
        _pending.append((host, ev, f"edge_index of {B} graphs x {n} nodes"))
    lay = GraphLayout("block", n, B, N, E, ei, rowmask, canonical_table(n, device), eid, bad)
    return _attach(edge_index, key, lay)


def is_canonical_graph(edge_index: torch.Tensor, n: int) -> bool:
    """Whether ONE graph's edge_index is the reference's canonical order
    (checked on the host for host tensors; device tensors only when they are
    the cached canonical tensor or carry a canonical layout: no round trip)."""
    if edge_index.dim() != 2 or edge_index.size(0) != 2 or edge_index.size(1) != n * (n - 1):
        return False
    if edge_index.device.type == "cpu":
        return bool(torch.equal(edge_index, canonical_edge_index(n, 1)))
    for _, lay in (getattr(edge_index, "_sv2n_layouts", None) or {}).values():
        if lay.kind == "canonical" and lay.n == n and lay.num_graphs == 1:
            return True
    return False


def declare_canonical(edge_index: torch.Tensor, num_nodes: int, n: int) -> GraphLayout:
    """The canonical layout of a batch its builder verified (``collate`` sets
    ``canonical_edges`` after checking every graph on the host): no analysis,
    the kernels never read edge_index."""
    N, n = int(num_nodes), int(n)
    if n < 1 or n > MAX_N or N % n != 0 or edge_index.size(1) != (N // n) * n * (n - 1):
        raise UnsupportedLayout(f"batch marked canonical does not hold {N // max(n, 1)} "
                                f"complete {n}-node graphs")
    key = (N, n)
    lay = _cached(edge_index, key)
    if lay is not None and lay.kind == "canonical":
        return lay
    lay = GraphLayout("canonical", n, N // n, N, edge_index.size(1), None, None,
                      canonical_table(n, edge_index.device))
    return _attach(edge_index, key, lay)


def analyze_edge_index(edge_index: torch.Tensor, num_nodes: int,
                       n: Optional[int] = None, deferred: bool = True) -> GraphLayout:
    """Classify ``edge_index`` (see module docstring); cached per tensor.
    ``n``: the graph size when known (``deferred``: analysed without a host
    round trip), or a candidate tried first by the synchronous analysis."""
    if edge_index.dim() != 2 or edge_index.size(0) != 2:
        raise ValueError("edge_index must have shape [2, E]")
    if edge_index.dtype != torch.long:
        raise TypeError("edge_index must be int64 (PyG convention)")
    key = (num_nodes, n)
    lay = _cached(edge_index, key)
    if lay is not None:
        return lay

    device = edge_index.device
    E = edge_index.size(1)
    N = int(num_nodes)
    if N <= 0:
        raise UnsupportedLayout("empty graph batch")
    if _pending:
        check_pending()
    if n is not None and deferred and device.type == "cuda":
        return _analyze_deferred(edge_index, N, int(n), key)

    # 1) block size
    cands = []
    if n is not None and deferred:
        cands = [int(n)]
    else:
        if n is not None:
            cands.append(int(n))
        if E > 0 and E % N == 0:
            guess = E // N + 1
            if N % guess == 0:
                cands.append(guess)
        cands += [k for k in range(2, MAX_N + 1) if N % k == 0 and k not in cands]
    src, dst = edge_index[0], edge_index[1]
    nb = None
    if E == 0:  # isolated nodes: any block size is exact; 1 needs no mask
        nb = int(n) if n is not None else 1
    else:
        lo = torch.minimum(src, dst).min()
        hi = torch.maximum(src, dst).max()
        if int(lo) < 0 or int(hi) >= N:
            raise ValueError("edge_index refers to nodes outside [0, num_nodes)")
        for k in cands:
            if k > MAX_N or N % k != 0:
                continue
            if bool(torch.equal(src // k, dst // k)):
                nb = k
                break
    if nb is None:
        raise UnsupportedLayout(
            f"graph batch is not a union of equal-size blocks of <= {MAX_N} nodes")
    B = N // nb

    # 2) canonical?
    E0 = nb * (nb - 1)
    canon = canonical_table(nb, device)
    if E == 0:  # isolated nodes only: every target keeps just its self loop
        rowmask = None if nb == 1 else torch.zeros(N * _words(nb), dtype=torch.int32,
                                                    device=device)
        lay = GraphLayout("canonical" if nb == 1 else "block", nb, B, N, 0, None, rowmask, canon)
        return _attach(edge_index, key, lay)
    if E == B * E0 and bool(torch.equal(edge_index, canonical_edge_index(nb, B, device))):
        lay = GraphLayout("canonical", nb, B, N, E, None, None, canon)
        return _attach(edge_index, key, lay)

    # 3) block: unique (target, source) pairs, optional bitmask
    keep = src != dst
    keyv = dst[keep] * nb + (src[keep] - (dst[keep] // nb) * nb)
    nk = int(keyv.numel())
    if nk and int(torch.unique(keyv).numel()) != nk:
        raise UnsupportedLayout("duplicate edges: the dense-block kernels need unique pairs")
    rowmask = None
    if nk != B * E0:
        rowmask = torch.zeros(N * _words(nb), dtype=torch.int32, device=device)
        if device.type != "cuda":
            raise UnsupportedLayout("the sv2n kernels need a ROCm device")
        _lib.check(_lib.load().sv2n_block_rowmask(edge_index.data_ptr(), E, N, nb,
                                                  rowmask.data_ptr(),
                                                  _lib.stream_handle(device)),
                   "sv2n_block_rowmask")
    eid = None
    if nb > SMALL_N:  # the tiled kernels address edge logits by edge id
        if device.type != "cuda":
            raise UnsupportedLayout("the sv2n kernels need a ROCm device")
        if E > 0x7FFFFFFF:
            raise UnsupportedLayout("more than 2^31 edges in one batch")
        eid = torch.full((N * nb,), -1, dtype=torch.int32, device=device)
        _lib.check(_lib.load().sv2n_block_eid(edge_index.data_ptr(), E, N, nb, eid.data_ptr(),
                                              _lib.stream_handle(device)), "sv2n_block_eid")
    lay = GraphLayout("block", nb, B, N, E, edge_index, rowmask, canon, eid)
    return _attach(edge_index, key, lay)
