"""GATModel.forward / backward replayed as hipGraphs (graphed.py) — the fast
path of the reference's own loop, 5_train_SpotV2Net.py:142-160, unchanged:
a new batch object per step, model(data), nn.MSELoss, zero_grad, backward,
torch.optim.Adam, loss.item()."""
import copy

import pytest
import torch

from helpers import assert_close

pytestmark = pytest.mark.gpu


def _model(dev, S=4, hidden=(16, 8), heads=4, seed=0, **kw):
    from spotv2net_amd import GATModel
    torch.manual_seed(seed)
    return GATModel(30 * S, 3 * S, heads, 1, list(hidden), concat_heads=True, **kw).to(dev)


def _fresh(data, n=30, canonical=False):
    """A new batch object with a new edge_index each step (what a DataLoader
    yields), graph size known (sv2n collate / PyG slice table); ``canonical``:
    marked as sv2n collate marks a batch of canonical-order graphs."""
    from spotv2net_amd import Batch
    extra = {"canonical_edges": True} if canonical else {}
    return Batch(x=data.x, edge_index=data.edge_index.clone(), edge_attr=data.edge_attr,
                 y_x=data.y_x, batch=data.batch, ptr=data.ptr, nodes_per_graph=n, **extra)


def _ref_loop(model, data, steps, lr=1e-3, canonical=False):
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    crit = torch.nn.MSELoss()
    losses = []
    for _ in range(steps):
        b = _fresh(data, canonical=canonical)
        loss = crit(model(b), b.y_x)
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(loss.item())
    return losses


@pytest.mark.parametrize("canonical", [False, True])
def test_reference_loop_replayed_equals_eager(dev, canonical):
    """The loop with graph replay (captured at step 2, replayed from step 3)
    gives the eager loop's losses and parameters bit for bit: the same
    kernels in the same order (block layout analysed per step, or the
    collate-verified canonical layout)."""
    from spotv2net_amd import synthetic_batch
    data = synthetic_batch(16, 4, seed=2, device=dev)
    m1 = _model(dev, seed=3)
    m2 = copy.deepcopy(m1)
    m2.graph_replay = False
    l1 = _ref_loop(m1, data, 6, canonical=canonical)
    l2 = _ref_loop(m2, data, 6, canonical=canonical)
    assert len(m1._graph_cache.entries) == 1 and m1._graph_cache.entries[
        next(iter(m1._graph_cache.entries))].g_bwd is not None
    assert l1 == l2
    for (n, p), (_, q) in zip(m1.named_parameters(), m2.named_parameters()):
        assert torch.equal(p, q), n


def _oracle_loop(ref, data, steps, grads_at=None):
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    losses = []
    for k in range(steps):
        loss = torch.nn.functional.mse_loss(ref(data), data.y_x)
        opt.zero_grad()
        loss.backward()
        if grads_at is not None and k == 0:
            grads_at.update({n: p.grad.detach().clone() for n, p in ref.named_parameters()})
        opt.step()
        losses.append(loss.item())
    return losses


def test_reference_loop_matches_oracle_after_3_steps(dev):
    """C2-shaped model (S 42, GAT [100, 50] x 4 heads concat, relu) through
    the reference loop on the replay path vs the PyG-semantics oracle running
    the same loop on the host.

    Step 1 — loss and every gradient — by the parity rule of tests/helpers.py
    (1e-5 of the fp32 oracle, or at least as close to the float64 oracle).
    Steps 2 and 3: losses within 1e-4 relative.  After an update the
    trajectories separate faster than fp32 rounding: a pre-activation within
    rounding of 0 takes ReLU's other branch (that node's whole contribution
    to a layer-0 gradient), and Adam's first steps move every weight by
    ~lr·g/|g|, so a rounding-level difference in a near-zero gradient entry is
    an lr-sized weight difference (MI355X: 1e-6 gradient error at step 1,
    2.8e-5 relative loss difference at step 3; fp32 vs float64 oracle 1e-6)."""
    from helpers import assert_parity, float64_twin, twin_model
    from spotv2net_amd import Data, synthetic_batch
    mine, ref = twin_model(seed=5154, num_node_features=1260, num_edge_features=126,
                           num_heads=4, output_node_channels=1, dim_hidden_layers=[100, 50],
                           concat_heads=True)
    ref64 = float64_twin(ref)
    mine = mine.to(dev)
    data = synthetic_batch(32, 42, seed=1234, device=dev)
    g_mine = {}
    opt = torch.optim.Adam(mine.parameters(), lr=1e-3)
    got = []
    for k in range(3):
        b = _fresh(data, canonical=True)
        loss = torch.nn.functional.mse_loss(mine(b), b.y_x)
        opt.zero_grad()
        loss.backward()
        if k == 0:
            g_mine = {n: p.grad.detach().clone() for n, p in mine.named_parameters()}
        opt.step()
        got.append(loss.item())
    cpu = synthetic_batch(32, 42, seed=1234)
    g32, g64 = {}, {}
    want = _oracle_loop(ref, cpu, 3, g32)
    cpu64 = Data(x=cpu.x.double(), edge_index=cpu.edge_index, edge_attr=cpu.edge_attr.double(),
                 y_x=cpu.y_x.double())
    want64 = _oracle_loop(ref64, cpu64, 3, g64)
    assert_parity(torch.tensor(got[0]), torch.tensor(want[0]), torch.tensor(want64[0]),
                  what="loss of step 1")
    for n in g32:
        assert_parity(g_mine[n], g32[n], g64[n], what=f"step-1 gradient of {n}")
    for k in (1, 2):
        assert abs(got[k] - want[k]) <= 1e-4 * abs(want[k]), (k + 1, got[k], want[k], want64[k])


def test_forward_awaiting_backward_is_not_overwritten(dev):
    """Two forwards before their backwards (gradient accumulation over two
    micro-batches): the second runs eagerly, both backwards are right."""
    from spotv2net_amd import synthetic_batch
    d1 = synthetic_batch(8, 4, seed=5, device=dev)
    d2 = synthetic_batch(8, 4, seed=6, device=dev)
    m1 = _model(dev, seed=7)
    m2 = copy.deepcopy(m1)
    m2.graph_replay = False
    for m in (m1, m2):
        for _ in range(3):  # capture (call 2) and replay (call 3) with d1's signature
            m(_fresh(d1)).sum().backward()
        m.zero_grad()
    for m in (m1, m2):
        a = m(_fresh(d1))
        b = m(_fresh(d1))      # same signature while a awaits its backward
        c = m(_fresh(d2))
        (a ** 2).sum().backward()
        (3 * b).sum().backward()
        (c ** 3).mean().backward()
    for (n, p), (_, q) in zip(m1.named_parameters(), m2.named_parameters()):
        assert torch.equal(p.grad, q.grad), n


def test_retained_backward_after_overwrite_raises(dev):
    from spotv2net_amd import synthetic_batch
    d = synthetic_batch(8, 4, seed=5, device=dev)
    m = _model(dev, seed=8)
    for _ in range(3):
        m(_fresh(d)).sum().backward()
    out = m(_fresh(d))
    loss = out.sum()
    loss.backward(retain_graph=True)
    m(_fresh(d)).sum().backward()   # replays the same graph: out's saved state is gone
    with pytest.raises(RuntimeError, match="overwritten"):
        loss.backward()


def test_inference_replay_and_autograd_grad(dev):
    """eval + no_grad calls replay a forward-only graph; torch.autograd.grad
    through a replayed training graph returns the eager gradients."""
    from spotv2net_amd import synthetic_batch
    d = synthetic_batch(12, 4, seed=9, device=dev)
    m1 = _model(dev, seed=10)
    m2 = copy.deepcopy(m1)
    m2.graph_replay = False
    m1.eval()
    m2.eval()
    with torch.no_grad():
        outs = [m1(_fresh(d)) for _ in range(3)]
        want = m2(_fresh(d))
    for o in outs:
        assert torch.equal(o, want)
    assert outs[0].data_ptr() != outs[2].data_ptr()  # fresh output per call
    m1.train()
    m2.train()
    for _ in range(3):
        g1 = torch.autograd.grad(m1(_fresh(d)).square().sum(), list(m1.parameters()))
    g2 = torch.autograd.grad(m2(_fresh(d)).square().sum(), list(m2.parameters()))
    for a, b in zip(g1, g2):
        assert torch.equal(a, b)
