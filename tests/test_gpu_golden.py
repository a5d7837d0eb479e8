"""GPU parity against the committed golden vectors (tests/golden/): the HIP
path behind GATConv / GATModel reproduces the oracle's fp32 forward output and
every gradient within the north-star tolerance (1e-5 fp32, helpers.TOL, with
the float64-anchored rule of helpers.assert_parity for cancellation-prone
gradients)."""
import os
import sys

import pytest
import torch

from helpers import assert_parity

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
import make_golden as mg  # noqa: E402

pytestmark = pytest.mark.gpu


def build_product(meta, arr, dev):
    from spotv2net_amd import GATConv, GATModel
    if meta["kind"] == "conv":
        m = GATConv(meta["in_channels"], meta["out_channels"], heads=meta["heads"],
                    concat=meta["concat"], negative_slope=meta.get("negative_slope", 0.2),
                    edge_dim=meta["edge_dim"])
    else:
        kw = {k: meta[k] for k in ("num_heads", "output_node_channels", "dim_hidden_layers",
                                   "concat_heads", "activation", "negative_slope",
                                   "standardize") if k in meta}
        m = GATModel(meta["num_node_features"], meta["num_edge_features"], **kw)
        m.train(meta["train"])
    sd = {k[2:]: torch.from_numpy(v) for k, v in arr.items() if k.startswith("p.")}
    m.load_state_dict(sd)
    m = m.to(dev)
    m._ei = torch.from_numpy(arr["edge_index"]).to(dev)
    return m


@pytest.mark.parametrize("name", mg.CASES)
def test_hip_path_matches_golden(name, dev):
    meta, arr = mg.load(name)
    m = build_product(meta, arr, dev)
    call = mg.conv_call if meta["kind"] == "conv" else mg.model_call
    t = lambda k: torch.from_numpy(arr[k]).to(dev)  # noqa: E731
    x = t("x")
    ea = t("edge_attr") if "edge_attr" in arr else None
    want_x = meta["kind"] == "conv"
    out, grads, gx = mg._run(m, call, x, ea, t("w_out"), want_x)
    assert_parity(out, t("out32"), t("out64"), what=f"{name} out")
    for k in [k[4:] for k in arr if k.startswith("g32.")]:
        assert k in grads, f"{name}: no gradient for {k}"
        assert_parity(grads[k], t("g32." + k), t("g64." + k), what=f"{name} d{k}")
    if want_x:
        assert_parity(gx, t("gx32"), t("gx64"), what=f"{name} dx")
