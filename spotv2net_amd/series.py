"""Matrix-series ingestion for the SpotV2Net data pipeline,
device-resident and PyG-free.

Restates, without HDF5 files in between (h5py is not part of this stack):

* ``matrix_series`` — reference 3_create_matrix_dataset.py
  ``generate_matrices`` (:15-83): per-pair covariance CSVs
  ``<root>/<covfolder>/<S1>_<S2>.csv`` and per-asset variance CSVs
  ``<root>/<varfolder>/<S>.csv`` (headerless, flattened column by column,
  :29-31/:39-41), symbols sorted (:46-50, asserted complete), matrix t has
  the variances on the diagonal and the covariances mirrored off it
  (:66-79); float64 [T, n, n].
* ``standardize`` — reference 4_standardize_data.py: one StandardScaler
  (population std; scale 1 for a zero-variance series, as sklearn) for the
  diagonal elements and one for the off-diagonal
  elements, fitted on matrices with index <= ``num_include`` (:42-43), applied
  to every matrix; returns the (mean, std) pairs the notebook uses to
  de-standardise predictions (6_results.ipynb cell 4 ``scalers``).

``load_series`` puts both series (vol and vol-of-vol) on the device, where
``data.WindowDataset`` slices training windows out of them with gathers.
"""
from __future__ import annotations

import os
from glob import glob
from typing import Dict, Tuple

import numpy as np
import torch

SOURCES = {"price": ("covol", "vol"), "vol": ("covol_of_vol", "vol_of_vol")}


def read_flat_csv(path: str) -> np.ndarray:
    """Headerless CSV flattened column by column (reference
    ``pd.concat([df[col] for col in df], ignore_index=True)``)."""
    a = np.loadtxt(path, delimiter=",", dtype=np.float64, ndmin=2)
    return a.reshape(-1, order="F")


def matrix_series(root: str, source: str = "price") -> Tuple[np.ndarray, list]:
    """[T, n, n] float64 matrices and the sorted symbol list."""
    covdir, vardir = SOURCES[source]
    covs: Dict[Tuple[str, str], np.ndarray] = {}
    symbols = set()
    for f in sorted(glob(os.path.join(root, covdir, "*.csv"))):
        pair = os.path.basename(f)[:-4]
        s1, s2 = pair.split("_")
        symbols.update((s1, s2))
        covs[(s1, s2)] = read_flat_csv(f)
    variances = {os.path.basename(f)[:-4]: read_flat_csv(f)
                 for f in sorted(glob(os.path.join(root, vardir, "*.csv")))}
    ordered = sorted(symbols | set(variances))
    missing = [s for s in ordered if s not in variances]
    if missing:  # reference :53 asserts every symbol has a variance series
        raise ValueError(f"no {vardir} series for {missing}")
    lengths = {len(v) for v in covs.values()} | {len(v) for v in variances.values()}
    if len(lengths) != 1:
        raise ValueError(f"series of different lengths: {sorted(lengths)}")
    T = lengths.pop()
    n = len(ordered)
    idx = {s: i for i, s in enumerate(ordered)}
    mats = np.full((T, n, n), np.nan)
    for s, v in variances.items():
        mats[:, idx[s], idx[s]] = v
    for (s1, s2), v in covs.items():
        mats[:, idx[s1], idx[s2]] = v
        mats[:, idx[s2], idx[s1]] = v
    return mats, ordered


def standardize(mats: np.ndarray, num_include: int) -> Tuple[np.ndarray, Dict[str, Tuple[float, float]]]:
    """Diagonal / off-diagonal standardisation with scalers fitted on
    matrices 0..num_include (inclusive, reference :42-43)."""
    T, n, _ = mats.shape
    eye = np.eye(n, dtype=bool)
    fit = mats[: min(T, num_include + 1)]
    diag = fit[:, eye]
    off = fit[:, ~eye]
    vm, vs = float(diag.mean()), float(diag.std())
    cm, cs = (float(off.mean()), float(off.std())) if off.size else (0.0, 1.0)
    # StandardScaler keeps a zero-variance feature as is (scale_ = 1)
    vs = vs if vs > 0 else 1.0
    cs = cs if cs > 0 else 1.0
    out = np.empty_like(mats)
    out[:, eye] = (mats[:, eye] - vm) / vs
    out[:, ~eye] = (mats[:, ~eye] - cm) / cs
    return out, {"Variance": (vm, vs), "Covariance": (cm, cs)}


def load_series(root: str, num_include: int, device=None):
    """(vol, volvol) standardised [T, n, n] fp32 tensors on ``device`` plus the
    variance (mean, std) of the vol series, for de-standardising predictions."""
    vol, sym = matrix_series(root, "price")
    volvol, sym2 = matrix_series(root, "vol")
    if sym != sym2:
        raise ValueError("vol and vol-of-vol series cover different symbols")
    vol_s, scal = standardize(vol, num_include)
    volvol_s, _ = standardize(volvol, num_include)
    t = lambda a: torch.from_numpy(a.astype(np.float32)).to(device)  # noqa: E731
    return t(vol_s), t(volvol_s), scal["Variance"], sym
