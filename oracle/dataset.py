"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restatement of ``CovarianceLaggedDataset.process`` (reference
utils/dataset.py:182-289) for in-memory matrices instead of HDF5 files
(h5py/natsort and PyG are absent here), following the reference's own numpy
idiom line by line so that the product's batched builder
(spotv2net_amd.data.window_batch) can be checked against it.
"""
from __future__ import annotations

import numpy as np
import torch


def lagged_windows(vol_mats, volvol_mats, seq_length, cut=0):
    """vol_mats, volvol_mats: sequences of [n, n] float64 arrays (the HDF5
    datasets in natsorted key order).  Returns a list of dicts with x,
    edge_index, edge_attr, y_x (torch tensors), like the PyG Data list."""
    out = []
    for i in range(len(vol_mats) - seq_length):                       # :200
        seq = []
        for j in range(seq_length):                                    # :202
            cov_matrix = np.array(vol_mats[i + j])                     # :204
            next_cov_matrix = np.array(vol_mats[i + j + 1])            # :205
            covol_matrix = np.array(volvol_mats[i + j])                # :207
            adj_matrix = covol_matrix.copy()                           # :212
            np.fill_diagonal(adj_matrix, 0)                            # :213
            mask = np.triu(np.ones_like(adj_matrix), k=1) > 0          # :216
            edge_index_upper = torch.tensor(np.argwhere(mask), dtype=torch.long).t().contiguous()
            edge_index_lower = edge_index_upper[[1, 0], :]
            edge_index = torch.cat([edge_index_upper, edge_index_lower], dim=1)
            variances = torch.tensor(np.diag(covol_matrix), dtype=torch.float)
            source_variances = variances[edge_index[0]]
            target_variances = variances[edge_index[1]]
            covariances = torch.tensor(adj_matrix[mask], dtype=torch.float)
            covariances = torch.cat([covariances, covariances])
            edge_attr = torch.stack([covariances, source_variances, target_variances], dim=1)
            x = torch.tensor(cov_matrix, dtype=torch.float)
            y_x = torch.tensor(np.diag(next_cov_matrix), dtype=torch.float)
            seq.append(dict(x=x, edge_index=edge_index, edge_attr=edge_attr, y_x=y_x))
        n = seq[0]["x"].shape[0]
        E = seq[-1]["edge_index"].shape[1]
        out.append(dict(
            x=torch.stack([d["x"] for d in seq], dim=2).reshape(n, -1),          # :279
            edge_index=seq[-1]["edge_index"],
            edge_attr=torch.stack([d["edge_attr"] for d in seq], dim=2).reshape(E, -1),
            y_x=seq[-1]["y_x"]))
    return out[cut:]


def lagged_windows_multi(vol_mats, volvol_mats, seq_length, future_steps, cut=0):
    """Restatement of ``CovarianceLaggedMultiOutputDataset.process``
    (reference utils/dataset.py:316-411): same window features as
    ``lagged_windows``; the target of the window's last step is the stack of
    the next ``future_steps`` vol diagonals, [n, F] (:385-390), flattened
    (:405, ``y_x.reshape(-1)``)."""
    out = []
    for i in range(len(vol_mats) - seq_length - future_steps + 1):     # :333
        seq = []
        for j in range(seq_length):                                    # :335
            cov_matrix = np.array(vol_mats[i + j])                     # :337
            covol_matrix = np.array(volvol_mats[i + j])                # :339
            adj_matrix = covol_matrix.copy()                           # :342
            np.fill_diagonal(adj_matrix, 0)                            # :343
            mask = np.triu(np.ones_like(adj_matrix), k=1) > 0          # :346
            edge_index_upper = torch.tensor(np.argwhere(mask), dtype=torch.long).t().contiguous()
            edge_index_lower = edge_index_upper[[1, 0], :]
            edge_index = torch.cat([edge_index_upper, edge_index_lower], dim=1)
            variances = torch.tensor(np.diag(covol_matrix), dtype=torch.float)
            source_variances = variances[edge_index[0]]
            target_variances = variances[edge_index[1]]
            covariances = torch.tensor(adj_matrix[mask], dtype=torch.float)
            covariances = torch.cat([covariances, covariances])
            edge_attr = torch.stack([covariances, source_variances, target_variances], dim=1)
            x = torch.tensor(cov_matrix, dtype=torch.float)
            ys = []
            for k in range(future_steps):                              # :385
                nxt = np.array(vol_mats[i + j + k + 1])
                ys.append(torch.tensor(np.diag(nxt), dtype=torch.float))
            y_x = torch.stack(ys, dim=1)                               # :390 [n, F]
            seq.append(dict(x=x, edge_index=edge_index, edge_attr=edge_attr, y_x=y_x))
        n = seq[0]["x"].shape[0]
        E = seq[-1]["edge_index"].shape[1]
        out.append(dict(
            x=torch.stack([d["x"] for d in seq], dim=2).reshape(n, -1),          # :402
            edge_index=seq[-1]["edge_index"],
            edge_attr=torch.stack([d["edge_attr"] for d in seq], dim=2).reshape(E, -1),
            y_x=seq[-1]["y_x"].reshape(-1)))                                    # :405
    return out[cut:]                                                           # :411
