"""CPU: the matrix-series pipeline (spotv2net_amd.series) restating
3_create_matrix_dataset.py generate_matrices and 4_standardize_data.py, on
the reference's own data file (tests/golden/processed_data/vol/AAPL.csv,
copied from the reference's processed_data/) and on a synthetic multi-asset
directory written by the test."""
import os

import numpy as np
import pytest

from spotv2net_amd import series

GOLD = os.path.join(os.path.dirname(__file__), "golden", "processed_data")


def test_reference_csv_flattens_column_by_column():
    a = np.loadtxt(os.path.join(GOLD, "vol", "AAPL.csv"), delimiter=",")
    flat = series.read_flat_csv(os.path.join(GOLD, "vol", "AAPL.csv"))
    assert a.shape == (14, 754) and flat.shape == (10556,)   # 10,556 matrices
    np.testing.assert_array_equal(flat[:14], a[:, 0])
    np.testing.assert_array_equal(flat[14:28], a[:, 1])


def _write(dirpath, name, arr):
    os.makedirs(os.path.dirname(os.path.join(dirpath, name)), exist_ok=True)
    np.savetxt(os.path.join(dirpath, name), arr, delimiter=",")


def test_matrix_series_layout(tmp_path):
    rng = np.random.default_rng(0)
    syms = ["MSFT", "AAPL", "JPM"]
    var = {s: rng.random((3, 5)) for s in syms}
    cov = {("AAPL", "JPM"): rng.random((3, 5)), ("JPM", "MSFT"): rng.random((3, 5)),
           ("AAPL", "MSFT"): rng.random((3, 5))}
    for s in syms:
        _write(tmp_path, f"vol/{s}.csv", var[s])
    for (a, b), v in cov.items():
        _write(tmp_path, f"covol/{a}_{b}.csv", v)
    mats, order = series.matrix_series(str(tmp_path), "price")
    assert order == sorted(syms) and mats.shape == (15, 3, 3)
    i = {s: k for k, s in enumerate(order)}
    t = 7  # column 2, row 1 of the 3 x 5 CSV
    for s in syms:
        assert mats[t, i[s], i[s]] == var[s][1, 2]
    for (a, b), v in cov.items():
        assert mats[t, i[a], i[b]] == mats[t, i[b], i[a]] == v[1, 2]
    os.remove(os.path.join(tmp_path, "vol", "JPM.csv"))
    with pytest.raises(ValueError):
        series.matrix_series(str(tmp_path), "price")


def test_standardize_matches_sklearn_scalers():
    from sklearn.preprocessing import StandardScaler
    rng = np.random.default_rng(1)
    mats = rng.random((20, 4, 4))
    mats = (mats + mats.transpose(0, 2, 1)) / 2
    out, sc = series.standardize(mats, num_include=11)
    eye = np.eye(4, dtype=bool)
    vsc = StandardScaler().fit(np.vstack([m[eye] for m in mats[:12]]).reshape(-1, 1))
    csc = StandardScaler().fit(np.vstack([m[~eye].reshape(-1, 1) for m in mats[:12]]))
    assert sc["Variance"] == pytest.approx((vsc.mean_[0], vsc.scale_[0]), rel=1e-12)
    assert sc["Covariance"] == pytest.approx((csc.mean_[0], csc.scale_[0]), rel=1e-12)
    np.testing.assert_allclose(out[:, eye], vsc.transform(mats[:, eye].reshape(-1, 1)).reshape(20, 4),
                               rtol=1e-12)


def test_real_aapl_series_standardizes():
    """The reference's AAPL vol file is a constant placeholder series
    (0.00024142): StandardScaler semantics give mean = that value, scale 1
    (zero variance), and an all-zero standardised series."""
    from sklearn.preprocessing import StandardScaler
    a = series.read_flat_csv(os.path.join(GOLD, "vol", "AAPL.csv")).reshape(-1, 1, 1)
    out, sc = series.standardize(a, num_include=7521)   # 4_standardize_data.py:19
    skl = StandardScaler().fit(a[:7522].reshape(-1, 1))
    assert sc["Variance"] == pytest.approx((skl.mean_[0], skl.scale_[0]), rel=1e-12)
    np.testing.assert_allclose(out.reshape(-1, 1), skl.transform(a.reshape(-1, 1)), atol=1e-12)
