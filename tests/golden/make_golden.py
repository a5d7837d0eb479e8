"""Generates the committed golden vectors in tests/golden/*.npz.

    python tests/golden/make_golden.py          (CPU, a few seconds)

The reference's own arithmetic (PyG 2.3.0 GATConv) is not importable here and
the reference holds no test vectors for this path, so parity
is unpinned: these vectors come from the oracle restatement
(oracle/pyg_gatconv.py), evaluated in fp32 and in float64, on the case grid
SURVEY.md §8c lists (B in {1,2,3}, n = 30, seq_length in {1,2}, H in {1,4},
C in {3,8}, concat on/off, relu/tanh/sigmoid, edge_attr None and 1-D, a
non-canonical edge order, a sparse graph with input self loops, multi-output
heads, BatchNorm standardisation).  They freeze the oracle (tests/test_golden.py
re-derives them on CPU) and are the fixture the GPU parity test
(tests/test_gpu_golden.py) checks the HIP path against.

Each .npz (numpy, no pickle) holds:
    meta        json string: kind ("conv" | "model"), constructor kwargs, n
    x, edge_index, [edge_attr], w_out        inputs and the loss weights
    p.<name>    every parameter / buffer of the state_dict (fp32)
    out32, out64                  forward output (fp32 oracle, float64 oracle)
    g32.<name>, g64.<name>        grads of loss = sum(out * w_out)
    gx32, gx64                    grad wrt x (conv cases only)
"""
from __future__ import annotations

import copy
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle.pyg_gatconv import OracleGATConv, OracleGATModel  # noqa: E402

N_NODES = 30


def canonical_edges(n, B):
    """CovarianceLaggedDataset order (utils/dataset.py:228-236): the row-major
    upper-triangle pairs (i<j) as (i->j), then the same pairs swapped."""
    iu = [(i, j) for i in range(n) for j in range(i + 1, n)]
    src = [i for i, j in iu] + [j for i, j in iu]
    dst = [j for i, j in iu] + [i for i, j in iu]
    one = torch.tensor([src, dst], dtype=torch.long)
    return torch.cat([one + g * n for g in range(B)], 1)


def graph(B, seed, keep_frac=1.0, shuffle=False, loops=False):
    g = torch.Generator().manual_seed(seed)
    ei = canonical_edges(N_NODES, B)
    if keep_frac < 1.0:
        ei = ei[:, torch.rand(ei.size(1), generator=g) < keep_frac]
    if loops:
        lp = torch.arange(0, B * N_NODES, 4).repeat(2, 1)
        ei = torch.cat([ei, lp], 1)
    if shuffle:
        ei = ei[:, torch.randperm(ei.size(1), generator=g)]
    return ei.contiguous()


class _D:
    def __init__(self, x, edge_index, edge_attr):
        self.x, self.edge_index, self.edge_attr = x, edge_index, edge_attr


CONV_CASES = [
    # name, B, S, kwargs, graph kwargs, edge_attr form ("2d" | "1d" | None)
    ("conv_b1_h1_c3_concat", 1, 1, dict(heads=1, out_channels=3, concat=True), {}, "2d"),
    ("conv_b2_h4_c8_mean", 2, 2, dict(heads=4, out_channels=8, concat=False), {}, "2d"),
    ("conv_b2_h4_c3_noedge", 2, 1, dict(heads=4, out_channels=3, concat=True), {}, None),
    ("conv_b2_h1_c8_edge1d", 2, 1, dict(heads=1, out_channels=8, concat=True), {}, "1d"),
    ("conv_b3_h4_c3_shuffled", 3, 1, dict(heads=4, out_channels=3, concat=True,
                                          negative_slope=0.1), dict(shuffle=True), "2d"),
    ("conv_b2_h4_c8_sparse_loops", 2, 2, dict(heads=4, out_channels=8, concat=True),
     dict(keep_frac=0.6, loops=True, shuffle=True), "2d"),
]

MODEL_CASES = [
    # name, B, S, GATModel kwargs (positional names of utils/models.py:62-73), train mode
    ("model_c2like_b2", 2, 2, dict(num_heads=4, output_node_channels=1, dim_hidden_layers=[8, 4],
                                   concat_heads=True, activation="relu"), True),
    ("model_1layer_tanh_b3", 3, 1, dict(num_heads=1, output_node_channels=1,
                                        dim_hidden_layers=[16], activation="tanh"), True),
    ("model_3layer_sigmoid_multiout_b1", 1, 1,
     dict(num_heads=2, output_node_channels=3, dim_hidden_layers=[6, 5, 4], concat_heads=True,
          activation="sigmoid", negative_slope=0.3), True),
    ("model_standardize_b2", 2, 1, dict(num_heads=4, output_node_channels=1,
                                        dim_hidden_layers=[8, 4], concat_heads=False,
                                        activation="relu", standardize=True), True),
]


def _inputs(B, S, seed, ea_form, gkw):
    g = torch.Generator().manual_seed(seed)
    ei = graph(B, seed + 1, **gkw)
    x = torch.randn(B * N_NODES, N_NODES * S, generator=g)
    D = 3 * S if ea_form == "2d" else 1
    ea = None
    if ea_form == "2d":
        ea = torch.randn(ei.size(1), D, generator=g)
    elif ea_form == "1d":
        ea = torch.randn(ei.size(1), generator=g)
    return x, ei, ea, D


def _run(module, call, x, ea, w, want_x_grad):
    x = x.clone().requires_grad_(want_x_grad)
    out = call(module, x, ea)
    (out * w).sum().backward()
    grads = {k: p.grad.detach().clone() for k, p in module.named_parameters()
             if p.grad is not None}
    return out.detach(), grads, (x.grad.detach().clone() if want_x_grad else None)


def _record(name, meta, x, ei, ea, w, module, call, want_x_grad):
    m64 = copy.deepcopy(module).double()
    out32, g32, gx32 = _run(module, call, x, ea, w, want_x_grad)
    out64, g64, gx64 = _run(m64, call, x.double(), None if ea is None else ea.double(),
                            w.double(), want_x_grad)
    arr = {"meta": np.array(json.dumps(meta)), "x": x.numpy(), "edge_index": ei.numpy(),
           "w_out": w.numpy(), "out32": out32.numpy(), "out64": out64.numpy()}
    if ea is not None:
        arr["edge_attr"] = ea.numpy()
    for k, v in module.state_dict().items():
        arr["p." + k] = v.detach().cpu().numpy()
    for k, v in g32.items():
        arr["g32." + k] = v.numpy()
    for k, v in g64.items():
        arr["g64." + k] = v.numpy()
    if want_x_grad:
        arr["gx32"], arr["gx64"] = gx32.numpy(), gx64.numpy()
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **arr)
    return arr


def conv_call(m, x, ea):
    return m(x, m._ei, ea)


def model_call(m, x, ea):
    return m(_D(x, m._ei, ea))


def make_all(verbose=True):
    made = []
    for i, (name, B, S, kw, gkw, ea_form) in enumerate(CONV_CASES):
        x, ei, ea, D = _inputs(B, S, 100 + i, ea_form, gkw)
        torch.manual_seed(7 + i)
        conv = OracleGATConv(N_NODES * S, edge_dim=(D if ea_form else None), **kw)
        with torch.no_grad():
            conv.bias.copy_(torch.randn_like(conv.bias) * 0.1)
        conv._ei = ei
        w = torch.randn(B * N_NODES, conv.bias.numel() if kw.get("concat", True) is False
                        else kw["heads"] * kw["out_channels"],
                        generator=torch.Generator().manual_seed(200 + i))
        if kw.get("concat", True) is False:
            w = w[:, :kw["out_channels"]].contiguous()
        meta = {"kind": "conv", "n": N_NODES, "in_channels": N_NODES * S,
                "edge_dim": (D if ea_form else None), "edge_attr": ea_form, **kw}
        _record(name, meta, x, ei, ea, w, conv, conv_call, True)
        made.append(name)
    for i, (name, B, S, kw, train) in enumerate(MODEL_CASES):
        x, ei, ea, D = _inputs(B, S, 300 + i, "2d", {})
        torch.manual_seed(11 + i)
        model = OracleGATModel(N_NODES * S, D, **kw)
        model.train(train)
        model._ei = ei
        w = torch.randn(B * N_NODES * kw["output_node_channels"],
                        generator=torch.Generator().manual_seed(400 + i))
        meta = {"kind": "model", "n": N_NODES, "num_node_features": N_NODES * S,
                "num_edge_features": D, "train": train, **kw}
        _record(name, meta, x, ei, ea, w, model, model_call, False)
        made.append(name)
    if verbose:
        tot = sum(os.path.getsize(os.path.join(HERE, m + ".npz")) for m in made)
        print(f"wrote {len(made)} fixtures, {tot / 1024:.0f} KiB")
    return made


def load(name):
    """(meta, arrays) of one fixture; numpy.load with allow_pickle=False."""
    with np.load(os.path.join(HERE, name + ".npz"), allow_pickle=False) as z:
        arr = {k: z[k] for k in z.files}
    return json.loads(str(arr.pop("meta"))), arr


CASES = [c[0] for c in CONV_CASES] + [c[0] for c in MODEL_CASES]

if __name__ == "__main__":
    make_all()
