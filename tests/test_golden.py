"""CPU: the committed golden vectors (tests/golden/, made by
tests/golden/make_golden.py from the oracle) are reproduced by the oracle in
fp32 and float64, and — for the single-layer cases — by the independent dense
float64 formulation (oracle/dense.py), so the fixture, the PyG-op restatement
and the math agree.  Parity with PyG itself is unpinned."""
import copy
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
import make_golden as mg  # noqa: E402


def build_oracle(meta, arr):
    from oracle.pyg_gatconv import OracleGATConv, OracleGATModel
    if meta["kind"] == "conv":
        m = OracleGATConv(meta["in_channels"], meta["out_channels"], heads=meta["heads"],
                          concat=meta["concat"], negative_slope=meta.get("negative_slope", 0.2),
                          edge_dim=meta["edge_dim"])
    else:
        kw = {k: meta[k] for k in ("num_heads", "output_node_channels", "dim_hidden_layers",
                                   "concat_heads", "activation", "negative_slope",
                                   "standardize") if k in meta}
        m = OracleGATModel(meta["num_node_features"], meta["num_edge_features"], **kw)
        m.train(meta["train"])
    sd = {k[2:]: torch.from_numpy(v) for k, v in arr.items() if k.startswith("p.")}
    m.load_state_dict(sd)
    m._ei = torch.from_numpy(arr["edge_index"])
    return m


def test_fixture_set_complete():
    for name in mg.CASES:
        assert os.path.exists(os.path.join(os.path.dirname(mg.__file__), name + ".npz")), name


@pytest.mark.parametrize("name", mg.CASES)
def test_oracle_reproduces_golden(name):
    meta, arr = mg.load(name)
    m = build_oracle(meta, arr)
    call = mg.conv_call if meta["kind"] == "conv" else mg.model_call
    x = torch.from_numpy(arr["x"])
    ea = torch.from_numpy(arr["edge_attr"]) if "edge_attr" in arr else None
    w = torch.from_numpy(arr["w_out"])
    want_x = meta["kind"] == "conv"
    for dt, tag, tol in ((torch.float32, "32", 2e-6), (torch.float64, "64", 1e-12)):
        mm = copy.deepcopy(m).to(dt)
        mm._ei = m._ei
        out, grads, gx = mg._run(mm, call, x.to(dt), None if ea is None else ea.to(dt),
                                 w.to(dt), want_x)
        np.testing.assert_allclose(out.numpy(), arr["out" + tag], rtol=tol, atol=tol)
        for k, g in grads.items():
            np.testing.assert_allclose(g.numpy(), arr[f"g{tag}.{k}"], rtol=tol, atol=tol,
                                       err_msg=k)
        assert {f"g{tag}.{k}" for k in grads} == {k for k in arr if k.startswith(f"g{tag}.")}
        if want_x:
            np.testing.assert_allclose(gx.numpy(), arr["gx" + tag], rtol=tol, atol=tol)


@pytest.mark.parametrize("name", [c for c in mg.CASES if c.startswith("conv_")])
def test_golden_matches_dense_formulation(name):
    from oracle.dense import gat_layer_dense
    meta, arr = mg.load(name)
    H, C = meta["heads"], meta["out_channels"]
    has_e = "edge_attr" in arr
    y, _ = gat_layer_dense(arr["x"], arr["edge_index"], arr.get("edge_attr"),
                           arr["p.lin_src.weight"], arr["p.att_src"], arr["p.att_dst"],
                           arr["p.lin_edge.weight"] if has_e else None,
                           arr["p.att_edge"] if has_e else None, arr["p.bias"], H, C,
                           meta["concat"], meta.get("negative_slope", 0.2), meta["n"])
    np.testing.assert_allclose(arr["out64"], y, rtol=1e-10, atol=1e-11)
    # the fp32 golden output is within the north-star tolerance of float64 truth
    assert np.abs(arr["out32"] - y).max() <= 1e-5 * max(1.0, np.abs(y).max())
