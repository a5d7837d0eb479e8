"""The torch.ops.sv2n operator boundary: schemas and fake
implementations (torch.library.opcheck), torch.compile over GATModel, and
the sync-free layout analysis with its deferred error."""
import pytest
import torch

from helpers import assert_close

pytestmark = pytest.mark.gpu

# schema + fake-impl checks.  opcheck's AOT-dispatch test also re-runs the op
# on RANDOMISED integer inputs (edge tables, masks), which these index-taking
# kernels trust; the ops carry no autograd formula (autograd lives in the
# fused nodes of stack.py), which its autograd tests expect.
UTILS = ("test_schema", "test_faketensor")


def _small(dev, B=3, S=2, n=30):
    from spotv2net_amd import synthetic_batch
    return synthetic_batch(B, S, n=n, seed=5, device=dev)


def test_opcheck_forward_ops(dev):
    """opcheck: schema, fake (meta) implementation and dispatcher registration
    of the forward operators on real inputs."""
    from spotv2net_amd import GATModel, library  # noqa: F401
    from spotv2net_amd.layout import analyze_edge_index
    ops = torch.ops.sv2n
    torch.manual_seed(0)
    m = GATModel(60, 6, 2, 1, [8, 4], concat_heads=True).to(dev)
    d = _small(dev)
    lay = analyze_edge_index(d.edge_index, d.x.shape[0])
    c0, c1 = m.gat_layers
    prep_args = ([c0.lin_src.weight, c1.lin_src.weight], [c0.att_src, c1.att_src],
                 [c0.att_dst, c1.att_dst], [c0.lin_edge.weight, c1.lin_edge.weight],
                 [c0.att_edge, c1.att_edge], [2, 2], [8, 4], 4, [False, True], True)
    torch.library.opcheck(ops.gat_prep, prep_args, test_utils=UTILS)
    waugs, planes, _, wf = ops.gat_prep(*prep_args)
    ea_args = (d.edge_attr, wf, None, lay.canon, 2, 2, 3, 30, False)
    torch.library.opcheck(ops.edge_logits, ea_args, test_utils=UTILS)
    aes = ops.edge_logits(*ea_args)
    pj = (d.x, planes[0], waugs[0], False, False)
    torch.library.opcheck(ops.project, pj, test_utils=UTILS)
    xs = ops.project(*pj)
    # the ReLU-masked store (sv2n_gemm_f32x3_relu) behind the optional relu_y
    ry = torch.randn(xs.shape, device=dev)
    torch.library.opcheck(ops.project, pj + (ry,), test_utils=UTILS)
    assert torch.equal(ops.project(*pj, ry), torch.where(ry > 0, xs, torch.zeros_like(xs)))
    assert aes[0].shape == (3 * 870, 2)  # canonical batch: edge-ordered logits
    att = (xs, aes[0], None, c0.bias, None, 1.0, 3, 30, 2, 8, True, 1, 0.2, True)
    torch.library.opcheck(ops.gat_attn_fwd, att, test_utils=UTILS)
    h = torch.randn(90, 4, device=dev)
    torch.library.opcheck(ops.head_fwd, (h, m.linear.weight, m.linear.bias), test_utils=UTILS)
    torch.library.opcheck(ops.head_mse_fwd, (h, m.linear.weight, m.linear.bias,
                                             torch.randn(90, device=dev)), test_utils=UTILS)


def test_opcheck_backward_ops(dev):
    from spotv2net_amd import library  # noqa: F401
    ops = torch.ops.sv2n
    g = torch.Generator().manual_seed(1)
    B, n, H, C = 2, 30, 2, 8
    ldx = (H * C + 2 * H + 3) // 4 * 4
    xs = torch.randn(B * n, ldx, generator=g).to(dev)
    ae = torch.randn(B, n, n, H, generator=g).to(dev)
    y, ps = ops.gat_attn_fwd(xs, ae, None, None, None, 1.0, B, n, H, C, True, 1, 0.2)
    dy = torch.randn_like(y)
    torch.library.opcheck(ops.gat_attn_bwd, (dy, y, xs, ps, None, 1.0, None, True, B, n, H, C,
                                             True, 1, 0.2), test_utils=UTILS)
    dxs, dae, dbp = ops.gat_attn_bwd(dy, y, xs, ps, None, 1.0, None, True, B, n, H, C, True, 1,
                                     0.2)
    # post-layer dropout fused into the attention (ABI 9): out == y masked and
    # scaled exactly as torch does it, and the backward masks dy first
    u = torch.rand(B * n, H * C, generator=g).to(dev)
    torch.library.opcheck(ops.gat_attn_fwd_post, (xs, ae, None, None, None, 1.0, u, 0.25, B, n,
                                                  H, C, True, 1, 0.2), test_utils=UTILS)
    y3, ps3, out3 = ops.gat_attn_fwd_post(xs, ae, None, None, None, 1.0, u, 0.25, B, n, H, C,
                                          True, 1, 0.2)
    assert torch.equal(y3, y) and torch.equal(ps3, ps)
    assert torch.equal(out3, y * ((u >= 0.25).to(torch.float32) * (1.0 / 0.75)))
    torch.library.opcheck(ops.gat_attn_bwd, (dy, y, xs, ps, None, 1.0, None, True, B, n, H, C,
                                             True, 1, 0.2, False, u, 0.25), test_utils=UTILS)
    dxs3, dae3, dbp3 = ops.gat_attn_bwd(dy, y, xs, ps, None, 1.0, None, True, B, n, H, C, True, 1,
                                        0.2, False, u, 0.25)
    dxs4, dae4, dbp4 = ops.gat_attn_bwd(dy * ((u >= 0.25).to(torch.float32) * (1.0 / 0.75)), y,
                                        xs, ps, None, 1.0, None, True, B, n, H, C, True, 1, 0.2)
    assert torch.equal(dxs3, dxs4) and torch.equal(dae3, dae4) and torch.equal(dbp3, dbp4)
    x = torch.randn(B * n, 12, generator=g).to(dev)
    W = torch.randn(H * C, 12, generator=g).to(dev)
    a_s = torch.randn(1, H, C, generator=g).to(dev)
    a_d = torch.randn(1, H, C, generator=g).to(dev)
    grads = [torch.zeros_like(W), torch.zeros_like(a_s), torch.zeros_like(a_d),
             torch.zeros(H * C, device=dev)]
    torch.library.opcheck(ops.gat_wgrad, (x, dxs, W, a_s, a_d, dbp, H, C, False, *grads),
                          test_utils=UTILS)
    ae_e = torch.randn(B * n * (n - 1), H, generator=g).to(dev)
    y2, ps2 = ops.gat_attn_fwd(xs, ae_e, None, None, None, 1.0, B, n, H, C, True, 1, 0.2, True)
    torch.library.opcheck(ops.gat_attn_bwd, (torch.randn_like(y2), y2, xs, ps2, None, 1.0, None,
                                             True, B, n, H, C, True, 1, 0.2, True),
                          test_utils=UTILS)
    lin = torch.nn.Linear(4, 1).to(dev)
    h = torch.randn(60, 4, device=dev)
    torch.library.opcheck(ops.head_bwd, (h, lin.weight, torch.randn(60, 1, device=dev),
                                         torch.zeros_like(lin.weight),
                                         torch.zeros_like(lin.bias)),
                          test_utils=UTILS)


@pytest.mark.parametrize("precision", ["f32", "bf16"])
def test_torch_compile_matches_eager(dev, precision):
    """torch.compile(GATModel) (inductor) on a batch whose layout is attached:
    the sv2n ops appear in the traced graph as custom ops (no graph break
    inside the GAT stack) and the forward / gradients equal eager.  bf16: the
    eager backward runs on two streams (stack.BWD_OVERLAP), the traced one
    on one."""
    import copy

    from spotv2net_amd import GATModel
    torch.manual_seed(2)
    m1 = GATModel(60, 6, 2, 1, [8, 4], concat_heads=True).to(dev).set_precision(precision)
    m2 = copy.deepcopy(m1)
    d = _small(dev)
    torch._dynamo.reset()
    explain = torch._dynamo.explain(m2)(d)
    cm = torch.compile(m2)
    out1 = m1(d)
    out2 = cm(d)
    assert_close(out2, out1, tol=1e-6, what="compiled forward")
    out1.sum().backward()
    out2.sum().backward()
    for (name, p), (_, q) in zip(m1.named_parameters(), m2.named_parameters()):
        assert_close(q.grad, p.grad, tol=1e-6, what=name)
    # the stack is one traceable region: breaks, if any, are outside sv2n ops
    for br in explain.break_reasons:
        assert "sv2n" not in str(br.reason), br


def test_layout_analysis_has_no_host_sync(dev):
    """A fresh edge_index per batch (the reference's PyG DataLoader loop,
    5_train_SpotV2Net.py:142-143) with a known graph size: forward and
    backward run with CUDA sync debugging set to error."""
    from spotv2net_amd import Batch, GATModel
    torch.manual_seed(3)
    m = GATModel(60, 6, 2, 1, [8, 4], concat_heads=True).to(dev)
    d = _small(dev, B=4)
    m(d).sum().backward()  # warm caches (canonical table, workspaces)
    fresh = Batch(x=d.x, edge_index=d.edge_index.clone(), edge_attr=d.edge_attr, y_x=d.y_x,
                  ptr=d.ptr, batch=d.batch, nodes_per_graph=30)
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")
    try:
        out = m(fresh)
        out.sum().backward()
    finally:
        torch.cuda.set_sync_debug_mode("default")
    assert_close(out, m(d), tol=1e-6, what="block path == canonical path")


def test_pyg_slice_table_counts_as_known_size(dev):
    """A PyG-style Batch (host-side ``_slice_dict`` with equal graph sizes, as
    PyG's collate writes it) takes the sync-free analysis too."""
    from spotv2net_amd import Batch, GATModel
    torch.manual_seed(3)
    m = GATModel(60, 6, 2, 1, [8, 4], concat_heads=True).to(dev)
    d = _small(dev, B=4)
    m(d).sum().backward()
    fresh = Batch(x=d.x, edge_index=d.edge_index.clone(), edge_attr=d.edge_attr, y_x=d.y_x,
                  ptr=d.ptr, batch=d.batch)
    fresh._slice_dict = {"x": torch.tensor([0, 30, 60, 90, 120])}
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")
    try:
        out = m(fresh)
    finally:
        torch.cuda.set_sync_debug_mode("default")
    assert_close(out, m(d), tol=1e-6, what="block path == canonical path")


def test_inferred_size_is_verified_synchronously(dev):
    """Graph size only inferred as N / num_graphs (no nodes_per_graph, no host
    slice table): the layout is checked before any compute, so a ragged batch
    (graphs of 20 and 40 nodes, N / num_graphs = 30) is never poisoned by the
    deferred check — it runs as one 60-node block and matches the oracle."""
    from helpers import twin_model
    from spotv2net_amd import Batch
    from spotv2net_amd.layout import canonical_edge_index
    mine, ref = twin_model(seed=9, num_node_features=6, num_edge_features=3, num_heads=2,
                           output_node_channels=1, dim_hidden_layers=[8, 4],
                           concat_heads=True)
    g = torch.Generator().manual_seed(4)
    ei = torch.cat([canonical_edge_index(20, 1), canonical_edge_index(40, 1) + 20], 1)
    x = torch.randn(60, 6, generator=g)
    ea = torch.randn(ei.size(1), 3, generator=g)
    ptr = torch.tensor([0, 20, 60])
    mine = mine.to(dev)
    out = mine(Batch(x=x.to(dev), edge_index=ei.to(dev), edge_attr=ea.to(dev),
                     ptr=ptr.to(dev)))
    want = ref(Batch(x=x, edge_index=ei, edge_attr=ea, ptr=ptr))
    assert torch.isfinite(out).all()
    assert_close(out, want, tol=1e-5, what="ragged batch")


def test_invalid_edges_poison_then_raise(dev):
    """Duplicate edges under the sync-free analysis: the forward returns NaN
    and the deferred check raises UnsupportedLayout."""
    from spotv2net_amd import Batch, GATModel, UnsupportedLayout
    from spotv2net_amd.layout import check_pending
    torch.manual_seed(4)
    m = GATModel(60, 6, 2, 1, [8, 4], concat_heads=True).to(dev)
    d = _small(dev, B=2)
    ei = d.edge_index.clone()
    ei[:, 5] = ei[:, 6]  # a repeated (target, source) pair
    bad = Batch(x=d.x, edge_index=ei, edge_attr=d.edge_attr, y_x=d.y_x, ptr=d.ptr,
                batch=d.batch, nodes_per_graph=30)
    out = m(bad)
    assert torch.isnan(out).all()
    with pytest.raises(UnsupportedLayout):
        check_pending(block=True)
    check_pending(block=True)  # reported once


def test_prep_bwd_edge_all_matches_per_layer(dev):
    """sv2n_gat_prep_bwd_edge_all (every layer's edge-fold backward in one
    launch) == sv2n_gat_prep_bwd_edge per layer, bit for bit (C2's two layers
    on one [126][8] fold gradient); opcheck of the op."""
    ops = torch.ops.sv2n
    g = torch.Generator(device="cpu").manual_seed(7)
    D, hp = 126, 8
    layers = [(4, 100), (4, 50)]
    dwf = torch.randn(D, hp, generator=g).to(dev)
    We = [torch.randn(H * C, D, generator=g).to(dev) for H, C in layers]
    ae = [torch.randn(H * C, generator=g).to(dev) for H, C in layers]
    gw1 = [torch.randn(H * C, D, generator=g).to(dev) for H, C in layers]
    ga1 = [torch.randn(H * C, generator=g).to(dev) for H, C in layers]
    gw2, ga2 = [t.clone() for t in gw1], [t.clone() for t in ga1]
    for l, (H, C) in enumerate(layers):
        ops.prep_bwd_edge(dwf, 4 * l, We[l], ae[l], H, C, gw1[l], ga1[l])
    ops.prep_bwd_edge_all(dwf, [0, 4], We, ae, [4, 4], [100, 50], gw2, ga2)
    for a, b in zip(gw1 + ga1, gw2 + ga2):
        assert torch.equal(a, b)
    torch.library.opcheck(ops.prep_bwd_edge_all,
                          (dwf, [0, 4], We, ae, [4, 4], [100, 50], [t.clone() for t in gw2],
                           [t.clone() for t in ga2]), test_utils=UTILS)
