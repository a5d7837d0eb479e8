"""CPU tests of the drop-in boundary: the C-ABI library loads and exports every
symbol include/sv2n.h declares (no compute calls), and the Python surface
matches the reference's GATModel / GATConv contract (ctor, state_dict keys,
init order) without needing a GPU."""
import os
import re

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_functions():
    txt = open(os.path.join(ROOT, "include", "sv2n.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\**\s+\**(sv2n_\w+)\s*\(", txt, re.M)))


def test_library_exports_every_header_symbol():
    from spotv2net_amd import _lib
    lib = _lib.load()
    names = _header_functions()
    assert len(names) >= 9, names
    for name in names:
        assert hasattr(lib, name), f"libsv2n.so lacks {name}"
    assert set(names) == set(_lib.EXPORTED_SYMBOLS), "ctypes table and header disagree"
    assert lib.sv2n_abi_version() == _lib.ABI_VERSION == 21
    assert b"invalid argument" in lib.sv2n_strerror(-1)


def test_argument_errors_without_gpu():
    """Argument validation happens before any HIP call, so it runs on CPU."""
    from spotv2net_amd import _lib
    lib = _lib.load()
    assert lib.sv2n_gat_attn_fwd(None, 8, None, 0, None, None, None, 1.0, None, None, None, 0.0,
                                 None, 1, 30, 4, 8, 1, 1, 0.2, None) == -1
    assert lib.sv2n_gemm_f32(1, 1, None, 4, None, 4, None, 4, 4, 4, 4, None, 0, None) == -1
    assert lib.sv2n_edge_logits_bwd_workspace(126, 8) == 1024 * 126 * 8
    # the fused head forward: NULL operands / unsupported shapes, before any HIP call
    assert lib.sv2n_gat_attn_fwd_head_mse(None, 8, None, 0, None, None, None, 1.0, None, None,
                                          None, 0.0, None, None, None, None, None, None, None,
                                          None, 0, 1, 30, 4, 8, 1, 1, 0.2, None) == -1
    assert lib.sv2n_gat_attn_fwd_head_mse_supported(512, 30, 4, 50, 0) == 1
    assert lib.sv2n_gat_attn_fwd_head_mse_supported(512, 40, 4, 50, 0) == 0  # n > 32
    assert lib.sv2n_gat_attn_fwd_head_mse_workspace(512, 4, 50, 0) == 512 * 52
    # the device dropout generator: NULL output / step
    assert lib.sv2n_dropout_uniform(None, 16, 1, None, 0, None) == -1
    # covariance-layout edge passes: NULL / unsupported shapes
    assert lib.sv2n_edge_logits_fwd_cv(None, 1, 30, 42, None, None, 16, None, 2, 4, None) == -1
    assert lib.sv2n_edge_logits_bwd_cv_workspace(42, 16) == 1024 * 126 * 16


def _ref_layer_dims(F, D, H, hidden, concat_heads):
    """reference utils/models.py:86-117 transcribed as (in, out, concat) triples."""
    L = len(hidden)
    out = [(F, hidden[0], False if L == 1 else concat_heads)]
    for i in range(L - 1):
        in_ch = hidden[i] * H if (concat_heads and H > 1) else hidden[i]
        out.append((in_ch, hidden[i + 1], False if i + 1 == L - 1 else concat_heads))
    return out


@pytest.mark.parametrize("hidden,H,concat", [([500], 6, True), ([100, 50], 4, True),
                                             ([100, 50, 25], 3, False), ([50, 50, 50], 1, True),
                                             ([600, 300, 150], 7, True)])
def test_gatmodel_stacking_and_keys(hidden, H, concat):
    from oracle.pyg_gatconv import OracleGATModel
    from spotv2net_amd import GATModel
    F, D = 30 * 42, 3 * 42
    torch.manual_seed(5154)
    m = GATModel(F, D, H, 1, hidden, concat_heads=concat)
    torch.manual_seed(5154)
    r = OracleGATModel(F, D, H, 1, hidden, concat_heads=concat)
    dims = _ref_layer_dims(F, D, H, hidden, concat)
    for conv, (i, o, c) in zip(m.gat_layers, dims):
        assert (conv.in_channels, conv.out_channels, conv.concat, conv.heads) == (i, o, c, H)
    sd, rsd = m.state_dict(), r.state_dict()
    assert list(sd.keys()) == list(rsd.keys())
    for k in sd:
        assert sd[k].shape == rsd[k].shape, k
        # same seed => same draws in the same order as the PyG restatement
        assert torch.equal(sd[k], rsd[k]), k
    assert sd["gat_layers.0.lin_src.weight"].data_ptr() == sd["gat_layers.0.lin_dst.weight"].data_ptr()


def test_state_dict_roundtrip_with_standardize():
    from spotv2net_amd import GATModel
    m = GATModel(12, 6, 2, 1, [8, 4], concat_heads=True, standardize=True)
    keys = set(m.state_dict())
    for k in ("bnorm_node.running_mean", "bnorm_edge.running_var", "linear.weight",
              "gat_layers.1.att_edge", "gat_layers.1.lin_edge.weight", "gat_layers.0.bias"):
        assert k in keys
    m2 = GATModel(12, 6, 2, 1, [8, 4], concat_heads=True, standardize=True)
    m2.load_state_dict(m.state_dict())


def test_unknown_activation_raises():
    from spotv2net_amd import GATModel
    with pytest.raises(ValueError):
        GATModel(12, 6, 2, 1, [8], activation="gelu")


def test_product_forward_refuses_cpu():
    from spotv2net_amd import GATModel, synthetic_batch
    m = GATModel(60, 6, 2, 1, [8])
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        m(synthetic_batch(2, 2))


def test_product_does_not_import_oracle():
    import ast
    pkg = os.path.join(ROOT, "spotv2net_amd")
    for fn in os.listdir(pkg):
        if fn.endswith(".py"):
            tree = ast.parse(open(os.path.join(pkg, fn)).read())
            for node in ast.walk(tree):
                if isinstance(node, (ast.Import, ast.ImportFrom)):
                    mod = getattr(node, "module", None) or ""
                    names = [a.name for a in node.names]
                    assert not mod.startswith("oracle") and not any(
                        n.startswith("oracle") for n in names), f"{fn} imports the oracle"
