"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py; parity unpinned).

Independent float64 numpy formulation of one PyG 2.3.0 GATConv layer on a
batch of dense-block graphs, written from the math rather than from PyG's op
sequence, to cross-check ``oracle.pyg_gatconv``:

for graph g, head h, target i, source j (j == i is the self loop):
    e[i,j]  = ea_row(j->i) · W_e,h · att_e,h             (edge term)
    e[i,i]  = mean_{j: j->i} ea_row(j->i) · W_e,h · att_e,h
    s[i,j]  = leaky(xs_j·att_s,h + xs_i·att_d,h + e[i,j])
    p[i,:]  = softmax over present j
    out_i,h = Σ_j p[i,j] xs_j,h ;  concat or mean over h ; + bias
"""
from __future__ import annotations

import numpy as np


def gat_layer_dense(x, edge_index, edge_attr, W, att_src, att_dst, W_edge, att_edge, bias,
                    heads, channels, concat, negative_slope, n):
    x = np.asarray(x, np.float64)
    W = np.asarray(W, np.float64)
    H, C = heads, channels
    N = x.shape[0]
    B = N // n
    xs = (x @ W.T).reshape(N, H, C)
    a_s = (xs * np.asarray(att_src, np.float64).reshape(1, H, C)).sum(-1)
    a_d = (xs * np.asarray(att_dst, np.float64).reshape(1, H, C)).sum(-1)
    ei = np.asarray(edge_index)
    present = np.zeros((N, n), bool)      # present[target row, local source]
    E_mat = np.zeros((N, n, H))           # edge logits
    if edge_attr is not None and W_edge is not None:
        ea = np.asarray(edge_attr, np.float64)
        if ea.ndim == 1:
            ea = ea[:, None]
        we = np.asarray(W_edge, np.float64).reshape(H, C, -1)
        ae = np.asarray(att_edge, np.float64).reshape(H, C)
        fold = np.einsum("hcd,hc->dh", we, ae)
        elog = ea @ fold                  # [E, H]
    else:
        elog = None
    for e in range(ei.shape[1]):
        s, t = int(ei[0, e]), int(ei[1, e])
        if s == t:
            continue
        j = s - (t // n) * n
        present[t, j] = True
        if elog is not None:
            E_mat[t, j] = elog[e]
    out = np.zeros((N, H, C))
    P = np.zeros((B, H, n, n))
    for t in range(N):
        g, i = divmod(t, n)
        mask = present[t].copy()
        cnt = mask.sum()
        loop_e = E_mat[t][mask].mean(0) if (cnt > 0 and elog is not None) else np.zeros(H)
        mask[i] = True
        for h in range(H):
            srow = a_s[g * n:(g + 1) * n, h] + a_d[t, h]
            erow = E_mat[t, :, h].copy()
            erow[i] = loop_e[h]
            srow = srow + erow
            srow = np.where(srow > 0, srow, srow * negative_slope)
            srow = np.where(mask, srow, -np.inf)
            pr = np.exp(srow - srow.max())
            pr = pr / pr.sum()
            P[g, h, i] = pr
            out[t, h] = pr @ xs[g * n:(g + 1) * n, h]
    y = out.reshape(N, H * C) if concat else out.mean(1)
    if bias is not None:
        y = y + np.asarray(bias, np.float64)
    return y, P
