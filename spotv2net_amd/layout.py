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
``UnsupportedLayout``.  Analysis runs on the device with torch ops and costs
one host synchronisation per new edge_index tensor.
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


def canonical_table(n: int, device: torch.device) -> torch.Tensor:
    key = ("table", n, str(device))
    if key not in _canon_cache:
        s, t = canonical_pairs(n)
        vals = [(ti << 8) | si for si, ti in zip(s, t)]
        _canon_cache[key] = torch.tensor(vals, dtype=torch.int32).to(torch.int16).to(device)
    return _canon_cache[key]


def canonical_edge_index(n: int, num_graphs: int = 1, device=None) -> torch.Tensor:
    """Batched canonical edge_index [2, B*n(n-1)] with PyG Batch node offsets."""
    device = torch.device(device) if device is not None else torch.device("cpu")
    key = ("ei", n, num_graphs, str(device))
    if key not in _canon_cache:
        s, t = canonical_pairs(n)
        one = torch.tensor([s, t], dtype=torch.long)
        off = (torch.arange(num_graphs, dtype=torch.long) * n).repeat_interleave(len(s))
        ei = one.repeat(1, num_graphs) + off.unsqueeze(0)
        ei = ei.to(device)
        if num_graphs * len(s) > 10_000_000:
            return ei  # do not pin very large batches in the cache
        _canon_cache[key] = ei
    return _canon_cache[key]


def _words(n: int) -> int:
    return (n + 31) // 32


def _attach(edge_index: torch.Tensor, key, layout: GraphLayout) -> GraphLayout:
    try:
        edge_index._sv2n_layout = (edge_index._version, key, layout)
    except (AttributeError, RuntimeError):
        pass
    return layout


def analyze_edge_index(edge_index: torch.Tensor, num_nodes: int,
                       n: Optional[int] = None) -> GraphLayout:
    """Classify ``edge_index`` (see module docstring); cached per tensor."""
    if edge_index.dim() != 2 or edge_index.size(0) != 2:
        raise ValueError("edge_index must have shape [2, E]")
    if edge_index.dtype != torch.long:
        raise TypeError("edge_index must be int64 (PyG convention)")
    key = (num_nodes, n)
    cached = getattr(edge_index, "_sv2n_layout", None)
    if cached is not None and cached[0] == edge_index._version and cached[1] == key:
        return cached[2]

    device = edge_index.device
    E = edge_index.size(1)
    N = int(num_nodes)
    if N <= 0:
        raise UnsupportedLayout("empty graph batch")

    # 1) block size
    cands = []
    if n is not None:
        cands = [int(n)]
    else:
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
