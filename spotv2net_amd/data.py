"""PyG-free graph containers and the SpotV2Net window-graph builder.

* ``Data`` / ``Batch`` / ``collate`` reproduce the PyG ``Data`` + DataLoader
  collation the reference relies on (5_train_SpotV2Net.py:90-91, :142-143):
  x rows concatenated, ``edge_index`` shifted by each graph's node offset,
  edge_attr and y_x concatenated, plus ``batch`` / ``ptr`` vectors.
  Real PyG ``Batch`` objects also work with GATModel (duck-typed).
* ``window_graph`` restates ``CovarianceLaggedDataset.process`` for one
  window (reference utils/dataset.py:200-282): node features are the rows of
  the S vol matrices (x[v, c*S+t] = vol_t[v, c]); edges are the canonical
  fully connected order; edge_attr[e, k*S+t] = (covol_t[u,v], var_t[src],
  var_t[tgt]) from the vol-of-vol matrix; y_x = diag(vol_{S}).
* ``window_batch`` builds B such windows on the device in one shot from a
  matrix series (the device-resident replacement of the per-window Python loop
  and the pickled InMemoryDataset cache).
* ``synthetic_series`` draws standardized symmetric matrices
  ((G+Gᵀ)/2, G ~ N(0,1)) matching 4_standardize_data.py's zero-mean data.
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch

from .layout import (canonical_edge_index, canonical_pairs, is_canonical_graph, mark_cov_var,
                     mark_cov_var_only)

_FIELDS = ("x", "edge_index", "edge_attr", "y_x")


class Data:
    """Minimal ``torch_geometric.data.Data`` stand-in with the fields the
    reference uses."""

    def __init__(self, x=None, edge_index=None, edge_attr=None, y_x=None, **kw):
        self.x = x
        self.edge_index = edge_index
        self.edge_attr = edge_attr
        self.y_x = y_x
        for k, v in kw.items():
            setattr(self, k, v)

    @property
    def num_nodes(self) -> int:
        return int(self.x.size(0))

    @property
    def num_edges(self) -> int:
        return int(self.edge_index.size(1))

    def to(self, device, non_blocking: bool = False):
        out = self.__class__.__new__(self.__class__)
        for k, v in self.__dict__.items():
            if isinstance(v, torch.Tensor):
                v = v.to(device, non_blocking=non_blocking)
            setattr(out, k, v)
        out.__dict__.pop("sv2n_layout", None)
        return out

    def __repr__(self) -> str:
        parts = [f"{k}={list(v.shape)}" for k, v in self.__dict__.items()
                 if isinstance(v, torch.Tensor)]
        return f"{self.__class__.__name__}({', '.join(parts)})"


def twin_only_x(data) -> bool:
    """Whether ``data.x`` is a ``WindowDataset.empty_batch(twin_only=True)``
    buffer: NaN, never written by ``fill`` — x exists only as its bf16 twin."""
    return bool(getattr(getattr(data, "x", None), "_sv2n_twin_only", False))


def bf16_twin(data) -> Optional[torch.Tensor]:
    """bf16(data.x) [N][K rounded up to 64] when the batch carries one written
    together with x (``WindowDataset.empty_batch(bf16_x=True)``) and x is
    still that tensor, unmodified by torch ops; else None."""
    xb = getattr(data, "_x_bf16", None)
    x = getattr(data, "x", None)
    if xb is None or x is None or getattr(data, "_x_bf16_of", None) != (x.data_ptr(), x._version):
        return None
    return xb


class Batch(Data):
    """A disjoint union of graphs (PyG ``Batch`` layout)."""

    @property
    def num_graphs(self) -> int:
        return int(self.ptr.numel() - 1)


def collate(graphs: Sequence[Data]) -> Batch:
    """PyG DataLoader collation: x/edge_attr/y_x concatenated, edge_index +=
    cumulative node count, ``batch`` and ``ptr`` added.  Equal graph sizes set
    ``nodes_per_graph``; when every graph's edge_index is the canonical order
    (checked here, on the host) the batch is marked ``canonical_edges`` and
    its layout needs no analysis on the device."""
    xs, eis, eas, ys, sizes = [], [], [], [], []
    off = 0
    for g in graphs:
        xs.append(g.x)
        eis.append(g.edge_index + off)
        if g.edge_attr is not None:
            eas.append(g.edge_attr)
        if g.y_x is not None:
            ys.append(g.y_x)
        sizes.append(g.num_nodes)
        off += g.num_nodes
    dev = graphs[0].x.device
    sizes_t = torch.tensor(sizes, dtype=torch.long, device=dev)
    ptr = torch.zeros(len(sizes) + 1, dtype=torch.long, device=dev)
    ptr[1:] = torch.cumsum(sizes_t, 0)
    b = Batch(x=torch.cat(xs, 0), edge_index=torch.cat(eis, 1),
              edge_attr=torch.cat(eas, 0) if eas else None,
              y_x=torch.cat(ys, 0) if ys else None,
              batch=torch.repeat_interleave(torch.arange(len(sizes), device=dev), sizes_t),
              ptr=ptr)
    if len(set(sizes)) == 1:
        b.nodes_per_graph = sizes[0]
        seen = set()
        canon = True
        for g in graphs:
            if id(g.edge_index) not in seen:
                if not is_canonical_graph(g.edge_index, sizes[0]):
                    canon = False
                    break
                seen.add(id(g.edge_index))
        if canon:
            b.canonical_edges = True
    return b


def window_graph(vol: torch.Tensor, volvol: torch.Tensor) -> Data:
    """One CovarianceLaggedDataset sample from S+1 consecutive matrices.

    vol, volvol: [S+1, n, n] (the window's S matrices plus the next one, whose
    diagonal is the target).  Restates utils/dataset.py:202-282 step by step."""
    S = vol.shape[0] - 1
    n = vol.shape[1]
    src, tgt = canonical_pairs(n)
    src_t = torch.tensor(src, dtype=torch.long)
    tgt_t = torch.tensor(tgt, dtype=torch.long)
    P = len(src) // 2
    xs, eas = [], []
    for t in range(S):
        cov = vol[t].float()
        covol = volvol[t]
        variances = torch.diagonal(covol).float()                  # :236
        cv = covol[src_t[:P], tgt_t[:P]].float()                  # adj_matrix[mask] :243
        cv = torch.cat([cv, cv])                                  # :245
        eas.append(torch.stack([cv, variances[src_t], variances[tgt_t]], dim=1))  # :247
        xs.append(cov)                                            # :254
    x = torch.stack(xs, dim=2).reshape(n, -1)                     # :279
    ea = torch.stack(eas, dim=2).reshape(len(src), -1)            # :281
    y = torch.diagonal(vol[S]).float()                            # :262
    return Data(x=x, edge_index=torch.stack([src_t, tgt_t]), edge_attr=ea, y_x=y)


def synthetic_series(T: int, n: int = 30, seed: int = 1234, device=None,
                     dtype=torch.float32) -> tuple[torch.Tensor, torch.Tensor]:
    """T standardized symmetric vol and vol-of-vol matrices [T, n, n]."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    G1 = torch.randn(T, n, n, generator=g, dtype=dtype)
    G2 = torch.randn(T, n, n, generator=g, dtype=dtype)
    V = (G1 + G1.transpose(1, 2)) / 2
    W = (G2 + G2.transpose(1, 2)) / 2
    if device is not None:
        V, W = V.to(device), W.to(device)
    return V, W


def window_batch(vol: torch.Tensor, volvol: torch.Tensor, starts: torch.Tensor,
                 seq_length: int, future_steps: int = 1) -> Batch:
    """Collated batch of the windows beginning at ``starts`` (window k uses
    matrices starts[k] .. starts[k]+S-1 and the target diag(vol[starts[k]+S])),
    built with gathers on the series' device; identical to
    ``collate([window_graph(...) for ...])``.

    ``future_steps`` = F > 1 gives CovarianceLaggedMultiOutputDataset's target
    (reference utils/dataset.py:385-390, :405): y_x[v*F + k] =
    diag(vol[starts+S+k])[v], k < F — the layout GATModel(output_node_channels=F)
    predicts (6_results.ipynb cell 52 reads it back as view(-1, 30, F))."""
    S = seq_length
    if future_steps < 1:
        raise ValueError("future_steps must be >= 1")
    n = vol.shape[1]
    dev = vol.device
    B = int(starts.numel())
    starts = starts.to(dev)
    tidx = starts.view(B, 1) + torch.arange(S, device=dev).view(1, S)       # [B, S]
    V = vol[tidx].float()                                                    # [B, S, n, n]
    W = volvol[tidx].float()
    x = V.permute(0, 2, 3, 1).reshape(B * n, n * S)                          # x[v, c*S+t]
    src, tgt = canonical_pairs(n)
    src_t = torch.tensor(src, dtype=torch.long, device=dev)
    tgt_t = torch.tensor(tgt, dtype=torch.long, device=dev)
    P = len(src) // 2
    cv = W[:, :, src_t[:P], tgt_t[:P]]                                       # [B, S, P]
    cv = torch.cat([cv, cv], dim=2)                                          # [B, S, E0]
    var = torch.diagonal(W, dim1=2, dim2=3)                                  # [B, S, n]
    ea = torch.stack([cv, var[:, :, src_t], var[:, :, tgt_t]], dim=2)       # [B, S, 3, E0]
    ea = ea.permute(0, 3, 2, 1).reshape(B * len(src), 3 * S)                 # ea[e, k*S+t]
    if future_steps == 1:
        y = torch.diagonal(vol[starts + S].float(), dim1=1, dim2=2).reshape(B * n)
    else:
        fidx = starts.view(B, 1) + S + torch.arange(future_steps, device=dev).view(1, -1)
        yk = torch.diagonal(vol[fidx].float(), dim1=2, dim2=3)                 # [B, F, n]
        y = yk.permute(0, 2, 1).reshape(B * n * future_steps)                  # y[v*F + k]
    ei = canonical_edge_index(n, B, dev)
    ptr = torch.arange(B + 1, device=dev) * n
    b = Batch(x=x.contiguous(), edge_index=ei, edge_attr=ea.contiguous(), y_x=y,
              batch=torch.arange(B, device=dev).repeat_interleave(n), ptr=ptr)
    b.nodes_per_graph = n
    mark_cov_var(b.edge_attr, S)  # written above in the reference's covariance layout
    return b


def synthetic_batch(num_graphs: int, seq_length: int, n: int = 30, seed: int = 1234,
                    device=None) -> Batch:
    """B independent windows (each from its own S+1 random matrices)."""
    T = num_graphs * (seq_length + 1)
    V, W = synthetic_series(T, n, seed, device)
    starts = torch.arange(num_graphs, device=V.device) * (seq_length + 1)
    return window_batch(V, W, starts, seq_length)


class WindowDataset:
    """Sliding windows over a matrix series, like CovarianceLaggedDataset
    (window i = matrices i .. i+S-1, target diag(vol[i+S]);
    utils/dataset.py:200-262), kept on the series' device; ``cut`` drops the
    first windows like the reference's ``data_list[8357:]`` (:287-288).
    ``future_steps`` > 1 is CovarianceLaggedMultiOutputDataset
    (utils/dataset.py:293-405): T - S - F + 1 windows (:333), F targets per
    node, the same cut (:411)."""

    def __init__(self, vol: torch.Tensor, volvol: torch.Tensor, seq_length: int, cut: int = 0,
                 future_steps: int = 1):
        self.vol, self.volvol, self.S = vol, volvol, seq_length
        self.future_steps = int(future_steps)
        last = vol.shape[0] - seq_length - self.future_steps + 1
        self.cut = int(cut)
        self.starts = torch.arange(cut, max(cut, last), device=vol.device)
        n = vol.shape[1]
        self.n = n
        dev = vol.device
        src, tgt = canonical_pairs(n)
        P = len(src) // 2
        # index vectors of the capturable gather (fill): no host->device copies
        self._src = torch.tensor(src, dtype=torch.long).to(dev)
        self._tgt = torch.tensor(tgt, dtype=torch.long).to(dev)
        self._up_s, self._up_t = self._src[:P], self._tgt[:P]
        self._arS = torch.arange(seq_length, device=dev)
        self._arF = torch.arange(self.future_steps, device=dev)
        # the series' diagonal volvol[t][v][v] as one [T][n] copy, built once:
        # the device window kernel reads it in runs instead of a line per element
        self.diag = torch.diagonal(volvol, dim1=1, dim2=2).contiguous() \
            if volvol.dtype == torch.float32 else None

    def empty_batch(self, batch_size: int, bf16_x: bool = False,
                    cov_var_only: bool = False, twin_only: bool = False) -> Batch:
        """Static device buffers of one batch of ``batch_size`` windows (the
        layout of ``batch``), for ``fill``: a hipGraph-captured train step
        reads the same tensors every replay.  ``bf16_x``: ``fill`` also
        writes bf16(x) (round to nearest even) beside x, which the bf16
        execution mode's layer-0 GEMMs read instead of rounding x themselves
        (``bf16_twin``).  ``cov_var_only``: ``fill`` writes of edge_attr only
        the columns the covariance-layout edge passes read
        (sv2n_window_gather_cv, ≈ 1/6 of its bytes) — for a consumer that
        reads it through those passes alone (``train.Fit`` when
        ``stack.cov_var_edges_only`` says so); any other edge path refuses the
        batch (``layout.check_full_edge_attr``).  ``twin_only`` (with
        ``bf16_x``): ``fill`` writes only the bf16 twin; x stays NaN and is
        marked (``twin_only_x``) — for a consumer whose layer-0 GEMMs read the
        twin alone (``train.Fit`` when ``stack.twin_only_ok`` says so; the
        stack refuses the batch on any path that would read x).  Ignored when
        no twin is made."""
        B, n, S = batch_size, self.n, self.S
        E0 = n * (n - 1)
        dev = self.vol.device
        b = Batch(x=torch.empty(B * n, n * S, device=dev),
                  edge_index=canonical_edge_index(n, B, dev),
                  edge_attr=torch.empty(B * E0, 3 * S, device=dev),
                  y_x=torch.empty(B * n * self.future_steps, device=dev),
                  batch=torch.arange(B, device=dev).repeat_interleave(n),
                  ptr=torch.arange(B + 1, device=dev) * n)
        b.nodes_per_graph = n
        if bf16_x and dev.type == "cuda":
            from .library import window_bf16x_supported
            if window_bf16x_supported(n, S, self.future_steps):
                b._x_bf16 = torch.zeros(B * n, (n * S + 63) // 64 * 64, device=dev,
                                        dtype=torch.bfloat16)
                if twin_only:
                    b.x.fill_(float("nan"))
                    b.x._sv2n_twin_only = True
                b._x_bf16_of = (b.x.data_ptr(), b.x._version)
        if cov_var_only and dev.type == "cuda" and self.vol.dtype == torch.float32 and \
                self.volvol.dtype == torch.float32 and 3 * S * (n + 1) * 4 <= 64 * 1024 and \
                self.future_steps <= 256:
            b._cov_var_only = True
        return b

    def fill(self, out: Batch, idx: torch.Tensor) -> None:
        """Gather the windows ``self.starts[idx]`` into ``out``'s buffers
        (from ``empty_batch(idx.numel())``), on the device, with no host
        synchronisation or host->device copy: capturable into a hipGraph.
        Same values as ``batch(idx)`` for ``idx`` in ``[0, len(self))``; an
        index outside that range (negative ones included: no Python-style
        wrap-around) gives NaN rows on the device path, the device-side error
        that needs no host round trip."""
        B, n, S, Fs = idx.numel(), self.n, self.S, self.future_steps
        P = self._up_s.numel()
        if self.vol.is_cuda and self.vol.dtype == torch.float32 and \
                self.volvol.dtype == torch.float32:
            # one sv2n::window_gather launch (include/sv2n.h sv2n_window_gather):
            # starts[idx] = cut + idx, added in the kernel (no gather launch);
            # an index past the windows names matrices past the series, a
            # negative one is refused by the kernel: NaN rows either way
            from . import library  # noqa: F401
            from .layout import canonical_table
            xb = bf16_twin(out)
            cv_only = bool(getattr(out, "_cov_var_only", False))
            torch.ops.sv2n.window_gather(self.vol.contiguous(), self.volvol.contiguous(),
                                         idx if idx.dtype == torch.long else idx.long(), S, Fs,
                                         canonical_table(n, self.vol.device), out.x,
                                         out.edge_attr, out.y_x, self.cut, self.diag, xb,
                                         cv_only, xb is not None and twin_only_x(out))
            mark_cov_var(out.edge_attr, S)
            if cv_only:
                mark_cov_var_only(out.edge_attr)
            return
        st = self.starts.index_select(0, idx)
        tidx = st.view(B, 1) + self._arS.view(1, S)                               # [B, S]
        V = self.vol[tidx]                                                        # [B, S, n, n]
        W = self.volvol[tidx]
        out.x.view(B, n, n, S).copy_(V.permute(0, 2, 3, 1))                       # x[v, c*S+t]
        ea = out.edge_attr.view(B, 2 * P, 3, S)                                   # ea[e, k*S+t]
        cv = W[:, :, self._up_s, self._up_t].permute(0, 2, 1)                     # [B, P, S]
        ea[:, :P, 0].copy_(cv)
        ea[:, P:, 0].copy_(cv)
        var = torch.diagonal(W, dim1=2, dim2=3).permute(0, 2, 1)                  # [B, n, S]
        ea[:, :, 1].copy_(var[:, self._src])
        ea[:, :, 2].copy_(var[:, self._tgt])
        fidx = st.view(B, 1) + S + self._arF.view(1, Fs)                          # [B, F]
        yk = torch.diagonal(self.vol[fidx], dim1=2, dim2=3)                       # [B, F, n]
        out.y_x.view(B, n, Fs).copy_(yk.permute(0, 2, 1))
        mark_cov_var(out.edge_attr, S)

    def __len__(self) -> int:
        return int(self.starts.numel())

    def batch(self, idx: torch.Tensor) -> Batch:
        return window_batch(self.vol, self.volvol, self.starts[idx.to(self.starts.device)],
                            self.S, self.future_steps)

    def loader(self, batch_size: int, shuffle: bool, generator: Optional[torch.Generator] = None,
               subset: Optional[torch.Tensor] = None, rank: int = 0, world_size: int = 1):
        """Batches of windows; with ``world_size > 1`` each rank walks its own
        shard (``shard_indices``), so every rank sees batch_size graphs per
        step (weak scaling).  Pass the same ``generator`` seed on every rank."""
        idx = subset if subset is not None else torch.arange(len(self))
        if shuffle:
            idx = idx[torch.randperm(idx.numel(), generator=generator)]
        if world_size > 1:
            idx = shard_indices(idx, rank, world_size)
        for k in range(0, idx.numel(), batch_size):
            yield self.batch(idx[k:k + batch_size])


def shard_indices(idx: torch.Tensor, rank: int, world_size: int) -> torch.Tensor:
    """torch.utils.data.DistributedSampler's partition (drop_last=False) of an
    already ordered index list: pad by wrapping to a multiple of world_size,
    then rank r takes positions r, r + world_size, ..."""
    n = idx.numel()
    total = -(-n // world_size) * world_size
    if total > n:
        reps = -(-(total - n) // max(n, 1))
        idx = torch.cat([idx, idx.repeat(reps)[:total - n]])
    return idx[rank:total:world_size]
