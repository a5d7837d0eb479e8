"""Edge passes for edge features in the reference's covariance layout
(utils/dataset.py:228-243, :279-282; sv2n_edge_logits_fwd_cv / _bwd_cv,
ABI 18): against the generic passes over every edge row on the same batch
(window_batch writes the layout), and a whole training step with the switch
on and off.  Tolerance: tests/helpers.py (1e-5 scaled)."""
import copy

import pytest
import torch

from helpers import assert_close

import spotv2net_amd  # noqa: F401  (registers torch.ops.sv2n)

pytestmark = pytest.mark.gpu


def _wfold(D, hp, dev, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(D, hp, generator=g) * 0.1).to(dev)


@pytest.mark.parametrize("B,S,n,L,H", [(64, 42, 30, 2, 4), (5, 2, 30, 1, 6), (3, 7, 9, 3, 5),
                                       (2, 40, 32, 2, 8),
                                       # past the backward's 512-graph grid; widest lags,
                                       # two-node graphs, odd n, 14 columns
                                       (600, 42, 30, 2, 4), (3, 64, 30, 3, 5), (6, 8, 2, 1, 3),
                                       (4, 30, 17, 1, 2), (2, 58, 24, 2, 7)])
def test_cov_var_logits_match_generic(dev, B, S, n, L, H):
    from spotv2net_amd import synthetic_batch
    from spotv2net_amd.layout import canonical_table, cov_var_seq_length
    b = synthetic_batch(B, S, n=n, seed=B + S, device=dev)
    assert cov_var_seq_length(b.edge_attr) == S
    canon = canonical_table(n, dev)
    hp = max(16, L * H)
    wf = _wfold(3 * S, hp, dev)
    ops = torch.ops.sv2n
    got = ops.edge_logits_cv(b.edge_attr, wf, canon, L, H, B, n)
    ref = ops.edge_logits(b.edge_attr, wf, None, canon, L, H, B, n, False)
    for l in range(L):
        assert_close(got[l], ref[l], what=f"ae layer {l}")
    daes = [torch.randn_like(r) for r in ref]
    dgot = ops.edge_logits_bwd_cv(b.edge_attr, canon, daes, H, B, n, hp)
    dref = ops.edge_logits_bwd(b.edge_attr, None, canon, daes, H, B, n, hp, False)
    assert_close(dgot[:, :L * H], dref[:, :L * H], what="dW~")
    assert torch.count_nonzero(dgot[:, L * H:]) == 0


def test_training_step_cov_var_on_off(dev):
    """C2-shaped model, B = 48: the step's loss and every gradient with the
    covariance-layout passes == with the generic passes."""
    from spotv2net_amd import GATModel, stack, synthetic_batch
    torch.manual_seed(3)
    m1 = GATModel(1260, 126, 4, 1, [100, 50], concat_heads=True).to(dev)
    m2 = copy.deepcopy(m1)
    data = synthetic_batch(48, 42, seed=4, device=dev)
    res = []
    for m, mode in ((m1, "on"), (m2, "off")):
        old = stack.COV_VAR_EDGES
        stack.COV_VAR_EDGES = mode
        try:
            loss = torch.nn.functional.mse_loss(m(data), data.y_x)
            loss.backward()
            res.append((loss.detach(), stack.LAST_PATH["cov_var"]))
        finally:
            stack.COV_VAR_EDGES = old
    assert res[0][1] is True and res[1][1] is False
    assert_close(res[0][0], res[1][0], tol=1e-6, what="loss")
    for (n, p), (_, q) in zip(m1.named_parameters(), m2.named_parameters()):
        assert_close(p.grad, q.grad, what=n)


def test_bwd_cv_switch_matches_generic(dev):
    """SV2N_COV_VAR_BWD=on (the backward's covariance-layout pass) gives the
    generic pass's edge gradients."""
    from spotv2net_amd import GATModel, stack, synthetic_batch
    torch.manual_seed(5)
    m1 = GATModel(120, 12, 4, 1, [16, 8], concat_heads=True).to(dev)
    m1.graph_replay = False
    m2 = copy.deepcopy(m1)
    data = synthetic_batch(16, 4, seed=2, device=dev)
    grads = []
    for m, bwd in ((m1, "on"), (m2, "off")):
        old = stack.COV_VAR_EDGES, stack.COV_VAR_BWD
        stack.COV_VAR_EDGES, stack.COV_VAR_BWD = "on", bwd
        try:
            torch.nn.functional.mse_loss(m(data), data.y_x).backward()
        finally:
            stack.COV_VAR_EDGES, stack.COV_VAR_BWD = old
        grads.append({k: p.grad for k, p in m.named_parameters()})
    for k in grads[0]:
        assert_close(grads[0][k], grads[1][k], what=k)


def test_inplace_write_drops_the_mark(dev):
    from spotv2net_amd import synthetic_batch
    from spotv2net_amd.layout import cov_var_seq_length
    b = synthetic_batch(2, 3, seed=1, device=dev)
    assert cov_var_seq_length(b.edge_attr) == 3
    b.edge_attr.mul_(2.0)
    assert cov_var_seq_length(b.edge_attr) is None


def test_c2_full_batch_cov_var_matches_oracle(dev):
    """C2 at the bench's B = 512 through the covariance-layout passes: the
    output and every gradient against the oracle (relu sides injected as in
    test_gpu_parity_full)."""
    from helpers import assert_parity, float64_twin, twin_model
    from spotv2net_amd import Batch, Data, stack, synthetic_batch
    from spotv2net_amd.layout import mark_cov_var
    from test_gpu_parity_full import _check_kinks, _relu_masks
    S = 42
    mine, ref = twin_model(seed=5154, num_node_features=30 * S, num_edge_features=3 * S,
                           num_heads=4, output_node_channels=1, dim_hidden_layers=[100, 50],
                           concat_heads=True)
    ref64 = float64_twin(ref)
    mine = mine.to(dev)
    data = synthetic_batch(512, S, seed=1234)
    gd = data.to(dev)
    # the device copy as its builder would hand it over: canonical edge order
    # and the covariance layout declared (.to() made new tensors)
    gd = Batch(x=gd.x, edge_index=gd.edge_index, edge_attr=mark_cov_var(gd.edge_attr, S),
               y_x=gd.y_x, batch=gd.batch, ptr=gd.ptr, nodes_per_graph=30, canonical_edges=True)
    old = stack.COV_VAR_EDGES
    stack.COV_VAR_EDGES = "on"
    try:
        masks = _relu_masks(mine, gd)
        ref.act_masks = masks
        ref64.act_masks = masks
        out = mine(gd)
        assert stack.LAST_PATH["cov_var"] is True
        torch.nn.functional.mse_loss(out, gd.y_x).backward()
    finally:
        stack.COV_VAR_EDGES = old
    d = Data(x=data.x, edge_index=data.edge_index, edge_attr=data.edge_attr)
    rout = ref(d)
    torch.nn.functional.mse_loss(rout, data.y_x).backward()
    r64 = ref64(Data(x=data.x.double(), edge_index=data.edge_index,
                     edge_attr=data.edge_attr.double()))
    torch.nn.functional.mse_loss(r64, data.y_x.double()).backward()
    _check_kinks(ref64, masks)
    assert_parity(out, rout, r64, what="forward")
    for (name, p), (_, q), (_, q64) in zip(mine.named_parameters(), ref.named_parameters(),
                                           ref64.named_parameters()):
        assert_parity(p.grad, q.grad, q64.grad, what=f"d{name}")
